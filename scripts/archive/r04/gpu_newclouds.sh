# r04: new-clouds wall-time breakdown (set_target / set_source / align), async covariance prep on and off
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-newclouds}; mkdir -p $O
MGICP_TRACE=1 timeout -k 10 300 python3 -u scripts/r04/new_clouds_trace.py > $O/async1.txt 2> $O/async1.err || { tail -5 $O/async1.err; exit 1; }
MGICP_TRACE=1 MGICP_ASYNC_COV=0 timeout -k 10 300 python3 -u scripts/r04/new_clouds_trace.py > $O/async0.txt 2> $O/async0.err || { tail -5 $O/async0.err; exit 1; }
SOURCE_FIRST=1 MGICP_TRACE=1 timeout -k 10 300 python3 -u scripts/r04/new_clouds_trace.py > $O/async1_sf.txt 2> $O/async1_sf.err || { tail -5 $O/async1_sf.err; exit 1; }
SOURCE_FIRST=1 MGICP_TRACE=1 MGICP_ASYNC_COV=0 timeout -k 10 300 python3 -u scripts/r04/new_clouds_trace.py > $O/async0_sf.txt 2> $O/async0_sf.err || { tail -5 $O/async0_sf.err; exit 1; }
cat $O/async1.txt $O/async0.txt $O/async1_sf.txt $O/async0_sf.txt

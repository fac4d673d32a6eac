# r06: phase traces of the reference's cold pair (fresh context, set_source, set_target, align, align) at C4 / C4F
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-trace}; mkdir -p $O
MGICP_TRACE=1 timeout -k 10 200 python scripts/r05/cold_pair.py 3 > $O/cold_c4.txt 2> $O/trace_c4.txt || { echo "cold failed"; tail -20 $O/trace_c4.txt; exit 1; }
cat $O/cold_c4.txt
MGICP_TRACE=1 MGICP_KNN_STATS=1 timeout -k 10 200 python scripts/r05/cold_pair.py 3 C4F > $O/cold_c4f.txt 2> $O/trace_c4f.txt || { echo "cold failed"; tail -20 $O/trace_c4f.txt; exit 1; }
cat $O/cold_c4f.txt

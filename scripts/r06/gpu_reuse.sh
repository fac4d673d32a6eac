# r06: reused-context diagnosis
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-reuse}; mkdir -p $O
timeout -k 10 300 python -u scripts/r06/reuse_diag.py 5000000 c4 > $O/reuse_c4.txt 2>&1 || { tail -20 $O/reuse_c4.txt; exit 1; }
cat $O/reuse_c4.txt
timeout -k 10 300 python -u scripts/r06/reuse_diag.py 5000000 same > $O/reuse_same.txt 2>&1 || { tail -20 $O/reuse_same.txt; exit 1; }
cat $O/reuse_same.txt

# r05: phase trace of GICPState cycles with the target cache (source grid guessed at set_source)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-trace}; mkdir -p $O
MGICP_TRACE=1 timeout -k 10 200 python scripts/r05/cold_pair.py 3 > $O/cold.txt 2> $O/trace.txt || { echo "cold failed"; tail -20 $O/trace.txt; exit 1; }
cat $O/cold.txt

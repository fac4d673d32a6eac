# r06: steady-state C4 align A/B of library builds (alternating, two rounds), then the listed-sweep GPU tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-steady}; mkdir -p $O
for round in 1 2; do
  for lib in ${LIBS:-libmgicp_prev.so libmgicp.so}; do
    MGICP_LIB_NAME=$lib timeout -k 10 200 python3 -u scripts/r06/steady_ab.py >> $O/steady.txt 2>&1 || { tail -20 $O/steady.txt; exit 1; }
    tail -1 $O/steady.txt
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gicp_gpu.py -m gpu -x -q -k "vlist or fused_compaction or lazy" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|Timeout" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log

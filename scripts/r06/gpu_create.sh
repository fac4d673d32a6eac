# r06: mgicp_create's phases (trace points) -> gpurun_out/r06/create*, then the engine GPU tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-create}; mkdir -p $O
for lib in ${LIBS:-libmgicp.so}; do
  MGICP_LIB_NAME=$lib MGICP_TRACE=1 timeout -k 10 120 python3 -u scripts/r06/create_trace.py > $O/out_$lib.txt 2> $O/trace_$lib.txt || { tail -20 $O/trace_$lib.txt; exit 1; }
  echo "== $lib"; cat $O/out_$lib.txt; grep -E 'create|\[py\]' $O/trace_$lib.txt
done
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gicp_gpu.py tests/test_abi.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|Timeout" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi

# r05: the xGMI row exchange on one GPU (several processes), then the rest of the distributed tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/xgmi}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -x -v --timeout 150 --timeout-method thread -m gpu -k "shared_rows or quits" -rP > $OUT/pytest_xgmi.log 2>&1 || { echo "xgmi tests failed"; grep -E "FAILED|Error|error" $OUT/pytest_xgmi.log | head -20; tail -30 $OUT/pytest_xgmi.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/pytest_xgmi.log | head -20
tail -1 $OUT/pytest_xgmi.log

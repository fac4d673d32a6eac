cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/xgmitime}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -x -v --timeout 150 --timeout-method thread -m gpu -k "shared_rows or quits" > $OUT/pytest_xgmi.log 2>&1 || { echo "xgmi tests failed"; tail -30 $OUT/pytest_xgmi.log; exit 1; }
tail -1 $OUT/pytest_xgmi.log
timeout -k 10 400 python3 scripts/r05/xgmi_time.py 200000 5 > $OUT/xgmi_time.txt 2>&1 || { echo "failed"; tail -20 $OUT/xgmi_time.txt; exit 1; }
cat $OUT/xgmi_time.txt

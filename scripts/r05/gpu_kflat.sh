# r05 A/B: the flattened ring-1 k-NN walk (MGICP_KNN_FLAT) -- per-cloud time, SQ counters, covariance bit-exactness
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-kflat}; mkdir -p $O
for v in "" _kflat; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 200 python scripts/r05/knn_time.py > $O/knn$v.txt 2>&1 || { echo "knn_time $v failed"; tail -20 $O/knn$v.txt; exit 1; }
  grep "knn_cov per" $O/knn$v.txt
done
MGICP_LIB_NAME=libmgicp_kflat.so timeout -k 10 400 python -u -m pytest tests/test_gicp_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "covariances or knn or logged or vlist or async or lazy" > $O/pytest_kflat.log 2>&1 || { echo "pytest kflat failed"; grep -E "FAILED|Error" $O/pytest_kflat.log | head; tail -20 $O/pytest_kflat.log; exit 1; }
tail -1 $O/pytest_kflat.log
for v in "" _kflat; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq$v -o run -- python3 scripts/r05/knn_time.py > $O/sq$v.log 2>&1 || { echo "sq $v failed"; tail -20 $O/sq$v.log; exit 1; }
  python3 scripts/pmc_kernels.py $O/sq$v > $O/sq_summary$v.txt 2>&1
  grep -A6 "knn_cov2_kernel<20>" $O/sq_summary$v.txt | head -7
done
find $O -name "*.csv" -size +20M -delete

# r05: k-NN parity tests, then the per-cloud time of each variant (knn_time.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/knn}
shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -k "covariances or knn or lazy or async or align_cube" > $OUT/pytest_knn.log 2>&1 || { echo "knn tests failed"; tail -60 $OUT/pytest_knn.log; exit 1; }
tail -1 $OUT/pytest_knn.log
for v in "$@"; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 200 python scripts/r05/knn_time.py > $OUT/knn$v.txt 2>&1 || { echo "knn_time $v failed"; tail -20 $OUT/knn$v.txt; exit 1; }
  grep -E "knn_cov per|\[knnb\]" $OUT/knn$v.txt | tail -2
done

# r05: the wave-staged k-NN kernel -- its parity tests, then per-cloud time vs the r04 kernel (variant kc2)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/knn}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -k "covariances or knn or lazy or async or align_cube" > $OUT/pytest_knn.log 2>&1 || { echo "knn tests failed"; tail -60 $OUT/pytest_knn.log; exit 1; }
tail -3 $OUT/pytest_knn.log
timeout -k 10 200 python scripts/r05/knn_time.py > $OUT/knn_time.txt 2>&1 || { echo "knn_time failed"; tail -20 $OUT/knn_time.txt; exit 1; }
MGICP_LIB_NAME=libmgicp_kc2.so timeout -k 10 200 python scripts/r05/knn_time.py >> $OUT/knn_time.txt 2>&1 || { echo "knn_time kc2 failed"; tail -20 $OUT/knn_time.txt; exit 1; }
cat $OUT/knn_time.txt

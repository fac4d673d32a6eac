# r05: k-NN covariance variants -- per-cloud time (knn_time.py) and the staging counters of the stats builds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/knnab}
shift
mkdir -p $OUT
for v in "$@"; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 200 python scripts/r05/knn_time.py > $OUT/knn_$v.txt 2>&1 || { echo "knn_time $v failed"; tail -20 $OUT/knn_$v.txt; exit 1; }
  grep -E "knn_cov per|\[knnb\]" $OUT/knn_$v.txt | tail -2
done

# A/B of the 1-NN query order (Morton vs grid-sorted) + work counters, then the GPU tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-qorder}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --gn-steps 3 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'gn', d['gn_mode']['value'], 'corr', round(k['correspond']['avg_ms'],3), 'cov', round(k['knn_cov']['avg_ms'],3))"
}
run morton
run grid MGICP_QUERY_ORDER=0
run morton_s16 MGICP_SRC_GRID_OCC=16
run morton2
MGICP_LIB_NAME=libmgicp_stats.so timeout -k 10 200 python bench.py --steps 1 --warmup 1 --gn-steps 0 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/stats.json 2> $OUT/stats.err && grep corr-stats $OUT/stats.err | head -3
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log

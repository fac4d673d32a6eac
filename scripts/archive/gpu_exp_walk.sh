# neighbour-graph walk seeding of the 1-NN sweeps: A/B over steps, work counters, GPU tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-walk}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 2 --gn-steps 10 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'gn', d['gn_mode']['value'], 'corr', round(k['correspond']['avg_ms'],3), 'gncorr', round(d['gn_mode']['kernels']['correspond']['avg_ms'],3), 'cov', round(k['knn_cov']['avg_ms'],3), 'prep', d['ms_to_converge_new_clouds_warm_process']['ms_prep'])"
}
run walk4
run walk0 MGICP_NN_WALK=0
run walk2 MGICP_NN_WALK=2
run walk8 MGICP_NN_WALK=8
run walk4b
MGICP_LIB_NAME=libmgicp_stats.so timeout -k 10 200 python bench.py --steps 1 --warmup 1 --gn-steps 0 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/stats.json 2> $OUT/stats.err && grep corr-stats $OUT/stats.err | head -3
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log

# A/B: branchless vs early-exit top-K insert in the k-NN covariance visitor (MGICP_KNN_INSERT_EARLY)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-insert}
mkdir -p $OUT
MGICP_LIB_NAME=libmgicp_early.so timeout -k 10 200 python -u -m pytest tests/test_gicp_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_early.log 2>&1 || { echo "early tests failed"; tail -20 $OUT/pytest_early.log; exit 1; }
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --gn-steps 0 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', 'cov', round(k['knn_cov']['avg_ms'],3), 'prep', d['ms_to_converge_new_clouds_warm_process']['ms_prep'], 'first', d['ms_to_converge_new_clouds_warm_process']['ms_wall'], 'it/s', d['value'])"
}
for r in 1 2; do
run base_$r || exit 1
run early_$r MGICP_LIB_NAME=libmgicp_early.so || exit 1
done

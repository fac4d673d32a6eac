# k-NN visitor candidate buffer: GPU tests (bit-exact covariances), then A/B of covariance time
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-knnbuf}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --gn-steps 0 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', 'cov', round(k['knn_cov']['avg_ms'],3), 'prep', d['ms_to_converge_new_clouds_warm_process']['ms_prep'], 'first', d['ms_to_converge_new_clouds_warm_process']['ms_wall'], 'frob', d['frob_vs_oracle_sample'])"
}
for r in 1 2; do
run buf4_$r
run buf0_$r MGICP_LIB_NAME=libmgicp_kb0.so
run buf2_$r MGICP_LIB_NAME=libmgicp_kb2.so
run buf8_$r MGICP_LIB_NAME=libmgicp_kb8.so
done

# tiled 1-NN: GPU parity tests, then C4 bench A/B over LDS budget / radius variants + per-sweep trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tile}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --cpu-sample 0 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -20 $OUT/bench_$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$name.json')); k=d['kernels']
print('$name', d['value'], 'corr', round(k['correspond']['avg_ms'],3), k['correspond'].get('search'), 'compact', round(k['compact_mahalanobis']['avg_ms'],3), 'fdf', round(k['fdf']['avg_ms'],4))"
  env "$@" MGICP_TRACE=1 timeout -k 10 300 python bench.py --cpu-sample 0 --steps 1 --warmup 1 2>&1 >/dev/null | grep "family 1" | tail -3 | tr '\n' ' '; echo
}
run tile MGICP_TILE_CORR=1
run batched MGICP_TILE_CORR=0
run nobatch MGICP_TILE_CORR=0 MGICP_LIB_NAME=libmgicp_nobatch.so
run w4 MGICP_TILE_CORR=0 MGICP_LIB_NAME=libmgicp_w4.so
echo done

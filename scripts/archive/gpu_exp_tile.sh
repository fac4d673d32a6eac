# tiled 1-NN: GPU parity tests, then C4 bench A/B (tiled vs global ring search)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tile}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for tc in 1 0; do
  MGICP_TILE_CORR=$tc timeout -k 10 300 python bench.py --cpu-sample 0 > $OUT/bench_tc$tc.json 2> $OUT/bench_tc$tc.err || { echo "bench failed"; tail -20 $OUT/bench_tc$tc.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_tc$tc.json')); k=d['kernels']
print('tc=$tc', d['value'], 'corr', k['correspond'], 'fdf', k['fdf']['avg_ms'], 'cov', k['knn_cov']['avg_ms'])"
done
echo done

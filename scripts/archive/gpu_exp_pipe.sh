cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pipe}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 2 --gn-steps 0 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'fdf', round(k['fdf']['avg_ms']*1e3,1), 'us', d['roofline']['achieved'])"
}
for r in 1 2; do
run pipe_$r
run nopipe_$r MGICP_FDF_PIPE=0
run pipe512_$r MGICP_FDF_BLOCKS=512
done
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log

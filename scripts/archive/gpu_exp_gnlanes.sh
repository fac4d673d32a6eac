cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-gnlanes}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --gn-steps 20 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); g=d['gn_mode']; print('$name', 'gn', g['value'], 'moments', round(g['kernels']['gn_moments']['avg_ms']*1e3,1), 'us', round(g['kernels']['gn_moments']['achieved_GBps'],0), 'GB/s')"
}
run lanes2
run lanes1 MGICP_GN_LANES=1
run lanes2b
run lanes1b MGICP_GN_LANES=1
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log

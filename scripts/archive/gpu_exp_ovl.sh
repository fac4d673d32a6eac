cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ovl}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 5 --warmup 2 --gn-steps 3 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], 'first', d['ms_to_converge_first'], d['ms_to_converge_new_clouds_warm_process'])"
}
for r in 1 2; do
run ovl_$r
run serial_$r MGICP_OVERLAP_COV=0
done

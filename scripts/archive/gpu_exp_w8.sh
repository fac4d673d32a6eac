cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-w8}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 2 --gn-steps 10 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'gn', d['gn_mode']['value'], 'corr', round(k['correspond']['avg_ms'],3), 'gncorr', round(d['gn_mode']['kernels']['correspond']['avg_ms'],3))"
}
for r in 1 2; do
run base_$r
run w8_$r MGICP_LIB_NAME=libmgicp_w8.so
done

# A/B of the fdf pass load policy: MGICP_FDF_HOT_MB (default-policy prefix; rest non-temporal)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-hot}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --gn-steps 0 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], round(d['kernels']['fdf']['avg_ms']*1e3,1), 'us fdf')"
}
run base
run nt_all MGICP_FDF_HOT_MB=0
run hot128 MGICP_FDF_HOT_MB=128
run hot192 MGICP_FDF_HOT_MB=192
run hot224 MGICP_FDF_HOT_MB=224
run hot192_fwd MGICP_FDF_HOT_MB=192 MGICP_FDF_ALT=0
run hot160_fwd MGICP_FDF_HOT_MB=160 MGICP_FDF_ALT=0
run nt_fwd MGICP_FDF_HOT_MB=0 MGICP_FDF_ALT=0
run base2
echo done

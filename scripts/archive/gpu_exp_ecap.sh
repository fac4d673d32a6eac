cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ecap}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --gn-steps 5 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'gn', d['gn_mode']['value'], 'corr', round(k['correspond']['avg_ms'],3), 'prep', d['ms_to_converge_new_clouds_warm_process']['ms_prep'], 'first', d['ms_to_converge_new_clouds_warm_process']['ms_wall'])"
}
for r in 1 2; do
run cap15_$r
run cap8_$r MGICP_LIB_NAME=libmgicp_ec8.so
run cap5_$r MGICP_LIB_NAME=libmgicp_ec5.so
done

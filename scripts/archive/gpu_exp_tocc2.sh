cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tocc2}
mkdir -p $OUT
run() {
  name=$1; shift
  env MGICP_SRC_GRID_OCC=12 "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 2 --gn-steps 10 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'gn', d['gn_mode']['value'], 'corr', round(k['correspond']['avg_ms'],3), 'gncorr', round(d['gn_mode']['kernels']['correspond']['avg_ms'],3), 'cov', round(k['knn_cov']['avg_ms'],3))"
}
for r in 1 2; do
run t12_$r
run t8_$r MGICP_GRID_OCC=8
run t10_$r MGICP_GRID_OCC=10
run t6_$r MGICP_GRID_OCC=6
done
echo done

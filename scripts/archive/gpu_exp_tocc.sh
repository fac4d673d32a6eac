# A/B of the target grid occupancy with the Morton query order (source grid fixed at 12)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tocc}
mkdir -p $OUT
run() {
  name=$1; shift
  env MGICP_SRC_GRID_OCC=12 "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --gn-steps 3 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'gn', d['gn_mode']['value'], 'corr', round(k['correspond']['avg_ms'],3), 'cov', round(k['knn_cov']['avg_ms'],3), 'prep', d['ms_to_converge_new_clouds_warm_process']['ms_prep'])"
}
run t12
run t6 MGICP_GRID_OCC=6
run t8 MGICP_GRID_OCC=8
run t16 MGICP_GRID_OCC=16
run t24 MGICP_GRID_OCC=24
run t32 MGICP_GRID_OCC=32
echo done

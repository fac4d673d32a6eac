# A/B of the source grid occupancy (source covariances + query order); target grid stays at 12
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-srcocc}
mkdir -p $OUT
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --gn-steps 3 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernels']; print('$name', d['value'], 'gn', d['gn_mode']['value'], 'corr', round(k['correspond']['avg_ms'],3), 'cov', round(k['knn_cov']['avg_ms'],3), 'first', d['ms_to_converge_new_clouds_warm_process'])"
}
run base
run s4 MGICP_SRC_GRID_OCC=4
run s6 MGICP_SRC_GRID_OCC=6
run s8 MGICP_SRC_GRID_OCC=8
run s16 MGICP_SRC_GRID_OCC=16
run base2
echo done

# r03: source-grid occupancy (the source grid serves only the source covariances' k-NN): C4 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-srcocc}; mkdir -p $O
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for rep in 1 2; do
  for v in 10 6 4 3; do
    MGICP_SRC_GRID_OCC=$v timeout -k 10 200 python3 $B > $O/b${v}_$rep.json 2> $O/b${v}_$rep.log || { tail -5 $O/b${v}_$rep.log; exit 1; }
    python3 - "$O/b${v}_$rep.json" "occ=$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
print(sys.argv[2], f"{d['value']:.1f} it/s", "knn_cov", json.dumps(k.get("knn_cov")), "first", json.dumps(d.get("ms_to_converge_first_detail")), "frob", d.get("frob_vs_oracle"))
PY
  done
done
echo done

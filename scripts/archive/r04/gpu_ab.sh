# r04 A/B: C4 bench lines of the default library against variant builds / env knobs, alternating, same box
# usage: gpu_ab.sh OUTNAME "ENV1" "ENV2" ...   (e.g. "MGICP_LIB_NAME=libmgicp_vb16.so" "MGICP_VLIST_CELL=0.6")
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-ab}; mkdir -p $O
shift
B="bench.py --steps 20 --warmup 5 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 ${AB_ARGS}"
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python3 $B > $O/b${i}_$rep.json 2> $O/b${i}_$rep.log || { echo "$cfg failed"; tail -5 $O/b${i}_$rep.log; exit 1; }
    python3 - "$O/b${i}_$rep.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
k = d.get("kernels", {})
nc = d.get("ms_to_converge_new_clouds_warm_process") or {}
print(f"{sys.argv[2]:42s} {d['value']:8.2f} it/s {d['ms_per_step']:7.3f} ms frac {r['frac']:.4f} "
      f"corr {k.get('correspond',{}).get('avg_ms',0)*1e3:6.1f} us compact {k.get('compact_mahalanobis',{}).get('avg_ms',0)*1e3:6.1f} us "
      f"new {nc.get('ms_wall')} (prep {nc.get('ms_prep')} loop {nc.get('ms_loop')}) frob {d.get('frob_vs_oracle')}")
PY
  done
done
echo done

# r04: C2 / C3 / C5 bench lines (short: no CPU legs) with the current engine
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-cfgs}; mkdir -p $O
for c in C2 C3 C5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 5 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 3 > $O/b_$c.json 2> $O/b_$c.log || { echo "$c failed"; tail -5 $O/b_$c.log; exit 1; }
  python3 - "$O/b_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; k = d.get("kernels", {})
print(f"{sys.argv[2]} {d['value']:9.2f} it/s {d['ms_per_step']:8.3f} ms/align  pass {r['avg_launch_ms']*1e3:7.2f} us  its {d['iterations_per_align']} passes {d['objective_passes_per_align']}  "
      f"corr {k.get('correspond',{}).get('avg_ms',0)*1e3:7.1f} us  gn {d['gn_mode']['value'] if d.get('gn_mode') else None}")
PY
done
echo done

# r03: 1-NN sweep kernel durations (sweeps 1/2/3 of a C4 align) over wave-kernel settings
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-corrsweep}; mkdir -p $O
shift
B="bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0"
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt$i -o run -- python3 $B > $O/b$i.json 2> $O/b$i.log || { echo "$cfg failed"; tail -5 $O/b$i.log; exit 1; }
  python3 - "$O/kt$i" "$cfg" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "correspond" in r["Kernel_Name"]]
d = d[-6:]
s = [sum(d[k::3]) / len(d[k::3]) for k in range(3)]
print(f"{sys.argv[2]:60s} sweeps us {s[0]:7.1f} {s[1]:7.1f} {s[2]:7.1f}  total {sum(s):7.1f}")
PY
  find $O/kt$i -name "*.csv" -delete
done
echo done

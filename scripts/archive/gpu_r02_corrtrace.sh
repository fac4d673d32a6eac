# per-sweep 1-NN timing in the C4 align (kernel trace, durations in launch order)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/corrtrace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 1 > $O/b.json 2> $O/log || { tail -20 $O/log; exit 1; }
f=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=[r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
out=[]
for r in rows:
    n=r['Kernel_Name']
    if 'correspond_kernel' in n or 'compact_kernel' in n or 'chunk_base' in n:
        out.append((n.split('(')[0].split('::')[-1], round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3,1)))
print(out)
PY
find $O -name "*kernel_trace.csv" -delete

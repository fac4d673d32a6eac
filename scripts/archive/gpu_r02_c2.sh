# C2 (100k <-> 100k): rate and kernel trace of one bench command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/c2; mkdir -p $O
timeout -k 10 300 python3 bench.py --config C2 --steps 20 --warmup 3 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/b.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'],d['objective_passes_per_align'],d['kernels'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --config C2 --steps 5 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/b2.json 2> $O/log || { tail -20 $O/log; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r['TotalDurationNs'])>2e5: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
f=$(find $O/kt -name "*kernel_trace.csv" | head -1); python3 - "$f" <<'PY'
import csv,sys
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:int(r['Start_Timestamp']))
fd=[r for r in rows if 'fdf_soa' in r['Kernel_Name']]
gaps=[(int(b['Start_Timestamp'])-int(a['End_Timestamp']))/1e3 for a,b in zip(fd,fd[1:])]
gaps=[g for g in gaps if g<200]
import statistics
print('fdf launches',len(fd),'median gap us',statistics.median(gaps) if gaps else None, 'median dur', statistics.median([(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in fd]))
PY
find $O -name "*kernel_trace.csv" -delete

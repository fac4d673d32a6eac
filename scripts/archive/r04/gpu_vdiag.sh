# r04: 1-NN cell-list diagnostics at C4 -- per-sweep list stats (stderr), rocprofv3 kernel stats of a short bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-vdiag}; mkdir -p $O
B="bench.py --steps 3 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --pass-bench 1 ${VDIAG_ARGS}"
MGICP_VLIST_STATS=1 timeout -k 10 300 python3 -u $B > $O/bench_stats.json 2> $O/bench_stats.err || { tail -30 $O/bench_stats.err; exit 1; }
grep -E "^\[vlist\]" $O/bench_stats.err | head -40
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $B > $O/b_rocprof.json 2> $O/kt.log || { tail -20 $O/kt.log; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats.csv
find $O -name "*kernel_trace.csv" -delete
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:22]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms tot')
"
echo done

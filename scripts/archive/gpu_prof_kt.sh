# kernel-trace stats of a short C4 bench (args: outdir, then env assignments)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-kt}; shift
mkdir -p $OUT
env "$@" timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > $OUT/bench.json 2> $OUT/kt.err || { echo "kernel trace failed"; tail -20 $OUT/kt.err; exit 1; }
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats.csv
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us avg', round(float(r['TotalDurationNs'])/1e6, 2), 'ms tot')
PY
find $OUT/kt -name "*.csv" -size +5M -delete
echo done

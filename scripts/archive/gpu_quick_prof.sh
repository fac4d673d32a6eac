# GPU tests, C4 bench and a kernel-trace summary (no PMC passes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench_C4.json 2> $OUT/bench_C4.err || { echo "bench failed"; tail -20 $OUT/bench_C4.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_C4.json')); print(d['value'], d['gn_mode']['value'], d['ms_to_converge_first'], d['ms_to_converge_new_clouds_warm_process'], d['frob_vs_oracle_sample'], d['gn_mode']['frob_vs_oracle_gn_sample'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/bench_under_kt.json 2> $OUT/kt.err || { echo "kernel trace failed"; tail -20 $OUT/kt.err; exit 1; }
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats.csv
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(r['Name'][:40].ljust(40), r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
find $OUT/kt -name "*.csv" -size +5M -delete

# logged k-NN kernel: exactness suites, fallback count and per-kernel split
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/knn3; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gicp_gpu.py tests/test_full_size_gpu.py tests/test_gicp_alignment.py tests/test_parity_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
MGICP_KNN_STATS=1 timeout -k 10 200 python -u $B > $O/b.json 2> $O/err || { tail $O/err; exit 1; }
grep "\[knn\]" $O/err | sort | uniq -c
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'knn' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY

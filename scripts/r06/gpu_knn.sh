# r06: k-NN split -- parity tests, A/B timing, rocprof kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-knn}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gicp_gpu.py -k "knn or covariances" -rP > $O/pytest_knn.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_knn.log | head; exit 1; }
tail -1 $O/pytest_knn.log
timeout -k 10 200 python -u scripts/r06/knn_ab.py 4 > $O/knn_ab.txt 2>&1 || { tail -20 $O/knn_ab.txt; exit 1; }
cat $O/knn_ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o knn -- python3 scripts/r06/knn_ab.py 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
python3 - <<PY
import csv, glob
for f in glob.glob("$O/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "knn" in r["Name"] or "finish" in r["Name"]:
            print(r["Name"][:60], r["Calls"], r["AverageNs"], r["TotalDurationNs"])
PY

# r06: k-NN split record -- rocprof kernel stats of knn_ab.py (both forms)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-knnprof}; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o knn -- python3 scripts/r06/knn_ab.py 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 - <<PY
import csv, glob
for f in glob.glob("$O/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "knn" in r["Name"] or "finish" in r["Name"]:
            print(r["Name"][:70], r["Calls"], r["AverageNs"], r["TotalDurationNs"])
PY

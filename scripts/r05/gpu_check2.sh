# r05 milestone check: GPU suite, smoke, k-NN variant times, C4 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/check}
shift
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -rP > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for v in "$@"; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 200 python scripts/r05/knn_time.py > $OUT/knn$v.txt 2>&1 || { echo "knn_time $v failed"; tail -20 $OUT/knn$v.txt; exit 1; }
  grep -E "knn_cov per|\[knnb\]" $OUT/knn$v.txt | tail -2
done
timeout -k 10 400 python bench.py > $OUT/bench_C4.json 2> $OUT/bench_C4.err || { echo "bench failed"; tail -20 $OUT/bench_C4.err; exit 1; }
python3 - $OUT/bench_C4.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms/step", d["ms_per_step"], "frob", d["frob_vs_oracle"], "frac", d["roofline"]["frac"])
print("cold_pair", json.dumps({k: v for k, v in d["cold_pair"].items() if k != "repeats"}))
print("new_clouds", json.dumps(d["ms_to_converge_new_clouds_warm_process"]))
print("c5", json.dumps(d["rooflines"]["fdf_52B_c5_past_infinity_cache"])[:400])
print("knn", json.dumps(d["rooflines"]["knn_cov"])[:300])
PY

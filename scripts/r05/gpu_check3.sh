# r05 milestone check: k-NN variant times, cold pair, GPU suite, smoke, C4 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/check}
shift
mkdir -p $OUT
for v in "$@"; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 200 python scripts/r05/knn_time.py > $OUT/knn$v.txt 2>&1 || { echo "knn_time $v failed"; tail -20 $OUT/knn$v.txt; exit 1; }
  grep -E "knn_cov per|\[knnb\]" $OUT/knn$v.txt | tail -2
done
timeout -k 10 200 python scripts/r05/cold_pair.py 4 > $OUT/cold.txt 2>&1 || { echo "cold failed"; tail -20 $OUT/cold.txt; exit 1; }
cat $OUT/cold.txt
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -rP > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_C4.json 2> $OUT/bench_C4.err || { echo "bench failed"; tail -20 $OUT/bench_C4.err; exit 1; }
python3 scripts/r05/show_bench.py $OUT/bench_C4.json

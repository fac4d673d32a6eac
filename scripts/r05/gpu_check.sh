# verify HEAD on the GPU: gpu tests, smoke, C4 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -rP > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_C4.json 2> $OUT/bench_C4.err || { echo "bench failed"; tail -20 $OUT/bench_C4.err; exit 1; }
cat $OUT/bench_C4.json
echo done

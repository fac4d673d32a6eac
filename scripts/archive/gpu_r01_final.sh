# round-1 final GPU check: gpu tests, smoke, C4 bench (+CPU baseline), C2/C3/C5 bench lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/final/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final/smoke.log; exit 1; }
for c in C4 C2 C3 C5; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/final/bench_$c.json 2> gpurun_out/final/bench_$c.err || { echo "bench $c failed"; tail -20 gpurun_out/final/bench_$c.err; exit 1; }
  echo "$c ok"
done
echo done

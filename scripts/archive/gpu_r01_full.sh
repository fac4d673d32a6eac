# round-1 GPU check: all gpu tests, smoke, bench (with CPU baseline), rocprofv3 kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_r01.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_r01.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r01.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r01.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r01.log; exit 1; }
cat gpurun_out/smoke_r01.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err || { echo "bench failed"; tail -20 gpurun_out/bench_r01.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r01 -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_r01_prof.json 2> gpurun_out/bench_r01_prof.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_r01_prof.err; exit 1; }
echo done

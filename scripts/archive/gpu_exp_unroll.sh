# regression tests, then bench + kernel trace with the unrolled candidate scans
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_7.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_7.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_7.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab5_unroll.json 2> gpurun_out/ab5_unroll.err || { echo "bench failed"; tail -5 gpurun_out/ab5_unroll.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r01c -o run -- python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_r01c_prof.json 2> gpurun_out/bench_r01c_prof.err || { echo "rocprof failed"; exit 1; }
echo done

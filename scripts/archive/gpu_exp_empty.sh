# regression tests, then A/B of the empty-space map (and the 256-block objective pass)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_6.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_6.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_6.log
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab4_$name.json 2> gpurun_out/ab4_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab4_$name.err; exit 1; }; }
run map MGICP_EMPTY_MAP=1
run nomap MGICP_EMPTY_MAP=0
run map2 MGICP_EMPTY_MAP=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r01b -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_r01b_prof.json 2> gpurun_out/bench_r01b_prof.err || { echo "rocprof failed"; exit 1; }
echo done

# regression tests, then A/B of alternating sweep direction (Infinity Cache reuse)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_8.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_8.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_8.log
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab6_$name.json 2> gpurun_out/ab6_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab6_$name.err; exit 1; }; }
run fwd MGICP_FDF_ALT=0
run alt MGICP_FDF_ALT=1
run fwd2 MGICP_FDF_ALT=0
run alt2 MGICP_FDF_ALT=1
run alt_b512 MGICP_FDF_ALT=1 MGICP_FDF_BLOCKS=512
echo done

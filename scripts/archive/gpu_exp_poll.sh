# regression tests, then A/B: host polling vs stream sync, events vs none in the timed region
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_9.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_9.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_9.log
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 $EXTRA > gpurun_out/ab7_$name.json 2> gpurun_out/ab7_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab7_$name.err; exit 1; }; }
run poll MGICP_POLL=1
run sync MGICP_POLL=0
EXTRA=--no-events run poll_noev MGICP_POLL=1
EXTRA=--no-events run sync_noev MGICP_POLL=0
run poll2 MGICP_POLL=1
echo done

# kernel preload at create + process-wide pinned uploader: GPU tests, traced bench, C4 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_upload2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_upload2.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_upload2.log
MGICP_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/trace_prep2.json 2> gpurun_out/trace_prep2.err || { echo "bench failed"; tail -5 gpurun_out/trace_prep2.err; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab11.json 2> gpurun_out/ab11.err || { echo "bench failed"; tail -5 gpurun_out/ab11.err; exit 1; }
echo done

# pinned pipelined upload + persistent build scratch: GPU tests, C4 bench x2, C5 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_upload.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_upload.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_upload.log
for r in a b; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab10_$r.json 2> gpurun_out/ab10_$r.err || { echo "bench failed"; tail -5 gpurun_out/ab10_$r.err; exit 1; }
done
MGICP_HOST_THREADS=16 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab10_t16.json 2> gpurun_out/ab10_t16.err || { echo "bench failed"; exit 1; }
timeout -k 10 400 python bench.py --config C5 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/ab10_c5.json 2> gpurun_out/ab10_c5.err || { echo "bench C5 failed"; tail -5 gpurun_out/ab10_c5.err; exit 1; }
echo done

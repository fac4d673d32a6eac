# experiment: regression tests, then grid occupancy sweep of the bench (no CPU baseline)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gicp_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu_2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_2.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_2.log
for occ in 3 6 12; do
  MGICP_GRID_OCC=$occ timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_occ_$occ.json 2> gpurun_out/bench_occ_$occ.err || { echo "bench occ=$occ failed"; tail -5 gpurun_out/bench_occ_$occ.err; exit 1; }
done
echo done

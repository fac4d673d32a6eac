# experiment: regression tests, then A/B of grid occupancy / fused finish / fdf grid
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gicp_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu_3.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_3.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_3.log
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab_$name.err; exit 1; }; }
run base MGICP_GRID_OCC=12 MGICP_FUSED_FINISH=0 MGICP_FDF_BLOCKS=2048
run fused2048 MGICP_GRID_OCC=12 MGICP_FUSED_FINISH=1 MGICP_FDF_BLOCKS=2048
run fused512 MGICP_GRID_OCC=12 MGICP_FUSED_FINISH=1 MGICP_FDF_BLOCKS=512
run sep512 MGICP_GRID_OCC=12 MGICP_FUSED_FINISH=0 MGICP_FDF_BLOCKS=512
run occ6 MGICP_GRID_OCC=6 MGICP_FUSED_FINISH=0 MGICP_FDF_BLOCKS=2048
run occ24 MGICP_GRID_OCC=24 MGICP_FUSED_FINISH=0 MGICP_FDF_BLOCKS=2048
run occ4 MGICP_GRID_OCC=4 MGICP_FUSED_FINISH=0 MGICP_FDF_BLOCKS=2048
echo done

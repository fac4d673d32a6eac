# A/B: 1-NN unroll 4 vs 8 (variant build), grid occupancy 8 / 12 / 16
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab8_$name.json 2> gpurun_out/ab8_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab8_$name.err; exit 1; }; }
MGICP_LIB_NAME=libmgicp_u8.so timeout -k 10 600 python -m pytest tests/test_gicp_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu_u8.log 2>&1 || { echo "pytest u8 failed"; tail -30 gpurun_out/pytest_gpu_u8.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_u8.log
run u4 MGICP_LIB_NAME=libmgicp.so
run u8 MGICP_LIB_NAME=libmgicp_u8.so
run u4_occ8 MGICP_LIB_NAME=libmgicp.so MGICP_GRID_OCC=8
run u4_occ16 MGICP_LIB_NAME=libmgicp.so MGICP_GRID_OCC=16
run u8_occ8 MGICP_LIB_NAME=libmgicp_u8.so MGICP_GRID_OCC=8
run u4b MGICP_LIB_NAME=libmgicp.so
echo done

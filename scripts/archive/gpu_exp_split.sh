# correspondence search split from Mahalanobis (fused into compaction); A/B of forced 8 waves/SIMD
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab9_$name.json 2> gpurun_out/ab9_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab9_$name.err; exit 1; }; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_split.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_split.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_split.log
run split MGICP_LIB_NAME=libmgicp.so
run w8 MGICP_LIB_NAME=libmgicp_w8.so
run split2 MGICP_LIB_NAME=libmgicp.so
run w8b MGICP_LIB_NAME=libmgicp_w8.so
echo done

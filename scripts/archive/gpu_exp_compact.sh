# regression tests, then A/B: compacted SoA objective pass vs in-place layout
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_4.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_4.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_4.log
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab2_$name.json 2> gpurun_out/ab2_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab2_$name.err; exit 1; }; }
run compact MGICP_FDF_COMPACT=1
run inplace MGICP_FDF_COMPACT=0
run compact_b1024 MGICP_FDF_COMPACT=1 MGICP_FDF_BLOCKS=1024
run compact_b256 MGICP_FDF_COMPACT=1 MGICP_FDF_BLOCKS=256
run compact2 MGICP_FDF_COMPACT=1
echo done

# r04: a selection of GPU tests (-k EXPR) and the new-clouds phase breakdown
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-quick2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "$2" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash scripts/r04/gpu_newclouds.sh ${1:-quick2}_nc

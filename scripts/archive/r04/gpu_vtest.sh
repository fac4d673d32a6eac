# r04: cell-list tests + diagnostics (the vlist GPU tests, C4/C4F parity, bench stats + rocprof)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-vtest}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gicp_gpu.py tests/test_parity_configs_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu -rP -k "vlist or C4 or correspondences or lattice or seeded" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
grep -E "^C[0-9]F?:" $O/pytest_gpu.log
bash scripts/r04/gpu_vdiag.sh ${1:-vtest}

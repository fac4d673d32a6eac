# r06: engine GPU tests + the C2/C2F/C4/C4F parity configs on the sketch-sized grid
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-sketcht}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gicp_gpu.py tests/test_parity_configs_gpu.py -m gpu -x -v -k "not C5 and not C3" --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|Timeout" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log

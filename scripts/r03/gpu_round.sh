# r03: full GPU suite, then the C4 A/B lines given as env settings, then sweep phases
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-round}; mkdir -p $O
shift
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
bash scripts/r03/gpu_ab.sh ${O#gpurun_out/r03/}/ab "$@"

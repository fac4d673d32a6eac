# stamped super partials to the host (no device total): tests, pass timing, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/hostsup; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_distributed.py tests/test_gicp_gpu.py tests/test_gicp_alignment.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -n "FAIL\|Error\|assert" $O/pytest.log | head -30; exit $rc; }
export PYTHONPATH=$GRAFT_REPO_ROOT
MGICP_PROF_STRIDE=1 timeout -k 10 120 python -u scripts/fdf_timing.py || exit 1
for i in 1 2; do timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/b$i.json 2> $O/err || { tail -30 $O/err; exit 1; }
python -c "import json;d=json.load(open('$O/b$i.json'));print(d['value'],d['ms_per_step'],d['kernels']['fdf'])"; done

# fixed reduction tree: distributed + engine suites, then a short bench for the objective-pass time
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/tree; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_distributed.py tests/test_gicp_gpu.py tests/test_gicp_alignment.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
[ $rc -ne 0 ] && { grep -n "FAIL\|Error\|error\|assert" $O/pytest.log | head -40; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 > $O/b.json 2> $O/err || { tail -30 $O/err; exit 1; }
python -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'],d['kernels'],d.get('frob_vs_oracle'))"

# 1-NN sweep: pointer-increment scans + seeded box search; exactness tests, A/B vs previous engine
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/nn; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gicp_gpu.py tests/test_full_size_gpu.py tests/test_parity_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="python -u bench.py --steps 20 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 5"
for lib in libmgicp.so libmgicp_noseedbox.so libmgicp_head.so libmgicp.so libmgicp_noseedbox.so libmgicp_head.so; do
 MGICP_LIB_NAME=$lib timeout -k 10 200 $B > $O/b_$lib.json 2> $O/err || { tail $O/err; exit 1; }
 python -c "import json;d=json.load(open('$O/b_$lib.json'));print('$lib',d['value'],d['ms_per_step'],d['kernels']['correspond'],d['gn_mode']['value'])"
done
MGICP_LIB_NAME=libmgicp_stats.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/stats.json 2> $O/stats.err; grep corr-stats $O/stats.err | head -3
echo done

# lazy-threshold logged k-NN vs the running-k-th form: exactness tests, covariance kernel time A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/knnlazy; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gicp_gpu.py tests/test_full_size_gpu.py tests/test_parity_configs_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -n "Error\|assert" $O/pytest.log | head; exit $rc; }
B="bench.py --steps 3 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events --pass-bench 0"
for L in libmgicp.so libmgicp_knn0.so libmgicp.so libmgicp_knn0.so; do
  MGICP_LIB_NAME=$L timeout -k 10 300 python -u $B > $O/b_$L.json 2> $O/b_$L.err || { tail -30 $O/b_$L.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$L.json')); r=d['rooflines']['knn_cov']; n=d['ms_to_converge_new_clouds_warm_process']; print('$L', 'knn_cov ms per cloud', round(r['avg_launch_ms'],3), 'frac', r['frac'], 'new clouds', n, 'it/s', d['value'])"
done

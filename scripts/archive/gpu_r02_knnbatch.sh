# logged k-NN with batched network insertion: exactness, then batch sweep
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/knnbatch; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gicp_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cov or knn or lattice" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
[ $rc -ne 0 ] && { grep -n "FAIL\|Error\|assert" $O/pytest.log | head -30; exit $rc; }
B="python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for b in 8 0 4 16 32 8; do MGICP_KNN_STATS=1 MGICP_KNN_BATCH=$b timeout -k 10 200 $B > $O/b$b.json 2> $O/err$b || { tail $O/err$b; exit 1; }
 python -c "import json;d=json.load(open('$O/b$b.json'));k=d['kernels']['knn_cov'];print('batch=$b', round(k['avg_ms']*k['count']/2,3),'ms/cloud', d['parity_full_size'] if 'parity_full_size' in d else '')"; grep "\[knn\]" $O/err$b | head -1; done

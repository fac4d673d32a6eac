# two-phase k-NN covariance kernel: bit-exactness suites, then A/B of the first-align prep
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/knn2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gicp_gpu.py tests/test_full_size_gpu.py tests/test_gicp_alignment.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for v in 1 0 1 0; do MGICP_KNN2=$v timeout -k 10 200 $B > $O/b$v.json 2> $O/err || { tail $O/err; exit 1; }
 python -c "import json;d=json.load(open('$O/b$v.json'));print('knn2=$v',d['value'],d['kernels']['knn_cov'],d['ms_to_converge_new_clouds_warm_process'])"; done
echo done

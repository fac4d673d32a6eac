# r03: register-list k-NN kernel (the logged kernel's hand-off, MGICP_KNN2=0 path) rows in guarded batches of 8
# (default build) vs 4-wide + tail (libmgicp_rl0.so): exactness, C4 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-knnrl}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gicp_gpu.py -k "covariances or logged_knn" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --steps 5 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for knn2 in 1 0; do
for rep in 1 2; do
  for v in libmgicp.so libmgicp_rl0.so; do
    MGICP_KNN2=$knn2 MGICP_LIB_NAME=$v timeout -k 10 200 python3 $B > $O/b_${knn2}_${v}_$rep.json 2> $O/b_${knn2}_${v}_$rep.log || { tail -5 $O/b_${knn2}_${v}_$rep.log; exit 1; }
    python3 - "$O/b_${knn2}_${v}_$rep.json" "knn2=$knn2 $v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
print(sys.argv[2], f"{d['value']:.1f} it/s", "knn_cov", json.dumps(k.get("knn_cov")))
PY
  done
done
done
echo done

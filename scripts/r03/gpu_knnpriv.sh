# r03: k-NN covariance log in LDS (default) vs private memory (MGICP_KNN_PRIV=1): exactness, then C4 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-knnpriv}; mkdir -p $O
MGICP_KNN_PRIV=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gicp_gpu.py -k "covariances or logged_knn" > $O/pytest_priv.log 2>&1 || { tail -20 $O/pytest_priv.log; exit 1; }
tail -3 $O/pytest_priv.log
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for rep in 1 2; do
  for v in 0 1; do
    MGICP_KNN_STATS=1 MGICP_KNN_PRIV=$v timeout -k 10 200 python3 $B > $O/b${v}_$rep.json 2> $O/b${v}_$rep.log || { tail -5 $O/b${v}_$rep.log; exit 1; }
    python3 - "$O/b${v}_$rep.json" "priv=$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
print(sys.argv[2], f"{d['value']:.1f} it/s", "knn_cov", json.dumps(k.get("knn_cov")), "first", json.dumps(d.get("ms_to_converge_first_detail")))
PY
  done
done
grep -h "left to the register" $O/b*_1.log | sort | uniq -c | head
echo done

# r03: k-NN near-first row order per lane (default) vs per wave (libmgicp_wo.so): exactness, divergence, C4 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-knnwo}; mkdir -p $O
MGICP_LIB_NAME=libmgicp_wo.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gicp_gpu.py -k "covariances or logged_knn" > $O/pytest_wo.log 2>&1 || { tail -20 $O/pytest_wo.log; exit 1; }
tail -2 $O/pytest_wo.log
MGICP_LIB_NAME=libmgicp_ph.so timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/ph.json 2> $O/ph.log || { tail -5 $O/ph.log; exit 1; }
grep "knn-div" $O/ph.log | sort | uniq -c
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for rep in 1 2; do
  for v in libmgicp.so libmgicp_wo.so; do
    MGICP_LIB_NAME=$v timeout -k 10 200 python3 $B > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.log || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python3 - "$O/b_${v}_$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
print(sys.argv[2], f"{d['value']:.1f} it/s", "knn_cov", json.dumps(k.get("knn_cov")), "first", json.dumps(d.get("ms_to_converge_first_detail")))
PY
  done
done
echo done

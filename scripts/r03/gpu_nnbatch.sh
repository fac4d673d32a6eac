# r03: 1-NN rows in guarded batches (variant builds libmgicp_nb4.so: 4 at 8 waves, libmgicp_nb8w6.so: 8 at 6
# waves) vs the default 4-wide + tail: exactness (sweep tests + full-size C4 parity in the bench), C4 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-nnbatch}; mkdir -p $O
for v in libmgicp_nb4.so libmgicp_nb8w6.so; do
  MGICP_LIB_NAME=$v timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gicp_gpu.py -k "correspondences or align or matched" > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for rep in 1 2; do
  for v in libmgicp.so libmgicp_nb4.so libmgicp_nb8w6.so; do
    MGICP_LIB_NAME=$v timeout -k 10 200 python3 $B > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.log || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python3 - "$O/b_${v}_$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
print(sys.argv[2], f"{d['value']:.1f} it/s {d['ms_per_step']:.3f} ms", "corr", json.dumps(k.get("correspond")), "frob", d.get("frob_vs_oracle"), d.get("frob_vs_oracle_sample"))
PY
  done
done
echo done

# resident server: odd waves stream first (stagger) vs all waves resident-first; parity + timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/stagger; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_distributed.py -m gpu -k "server_forms or resident" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -n "Error\|assert" $O/pytest.log | head; exit $rc; }
for L in libmgicp.so libmgicp_stag0.so libmgicp.so libmgicp_stag0.so; do
  MGICP_LIB_NAME=$L timeout -k 10 200 python -u scripts/srv_timing.py > $O/t_$L.json 2> $O/t_$L.err || { tail -20 $O/t_$L.err; exit 1; }
  echo "$L $(cat $O/t_$L.json)"
done
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events --pass-bench 0"
for L in libmgicp.so libmgicp_stag0.so libmgicp.so libmgicp_stag0.so; do
  MGICP_LIB_NAME=$L timeout -k 10 300 python -u $B > $O/b_$L.json 2> $O/b_$L.err || { tail -30 $O/b_$L.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$L.json')); print('$L', d['value'], d['ms_per_step'])"
done

# resident server variants (register groups 3 default / 4 / 2): pass timing, parity test, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/srv3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -k resident -x -q --timeout 240 --timeout-method thread > $O/pytest_resident.log 2>&1
rc=$?; tail -2 $O/pytest_resident.log; [ $rc -ne 0 ] && exit $rc
for L in libmgicp.so libmgicp_srv4.so libmgicp_srv2.so; do
  MGICP_LIB_NAME=$L timeout -k 10 200 python -u scripts/srv_timing.py > $O/t_$L.json 2> $O/t_$L.err || { tail -20 $O/t_$L.err; exit 1; }
  echo "$L $(cat $O/t_$L.json)"
done
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --no-events"
MGICP_PASS_TIMES=1 timeout -k 10 300 python -u $B > $O/b_on.json 2> $O/b_on.err || { tail -30 $O/b_on.err; exit 1; }
grep "pass-times" $O/b_on.err | tail -2
python3 -c "
import json
d=json.load(open('$O/b_on.json')); print('bench', d['value'], d['ms_per_step'])"

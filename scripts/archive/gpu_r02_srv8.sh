# resident server shapes: 4 waves (whole chunk in registers) vs 8 waves per CU; parity + timing + bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/srv8; mkdir -p $O
for W in 8 4; do
  MGICP_SRV_WAVES=$W timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -k resident -x -q --timeout 240 --timeout-method thread > $O/pytest_resident_$W.log 2>&1
  rc=$?; tail -1 $O/pytest_resident_$W.log; [ $rc -ne 0 ] && exit $rc
  MGICP_SRV_WAVES=$W timeout -k 10 200 python -u scripts/srv_timing.py > $O/t_$W.json 2> $O/t_$W.err || { tail -20 $O/t_$W.err; exit 1; }
  echo "waves $W $(cat $O/t_$W.json)"
done
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events --pass-bench 0"
for W in 8 4 8 4; do
  MGICP_SRV_WAVES=$W timeout -k 10 300 python -u $B > $O/b_$W.json 2> $O/b_$W.err || { tail -30 $O/b_$W.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$W.json')); print('waves $W', d['value'], d['ms_per_step'])"
done
for C in C2 C3; do
  timeout -k 10 300 python -u $B --config $C > $O/b_$C.json 2> $O/b_$C.err || { tail -30 $O/b_$C.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$C.json')); print('$C', d['value'], d['ms_per_step'])"
done

# resident server + host-row totals: parity tests, pass timing, bench A/B (host rows on/off, server off)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/srv4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_distributed.py tests/test_gicp_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_quick.log 2>&1
rc=$?; tail -2 $O/pytest_quick.log; [ $rc -ne 0 ] && { grep -n "Error\|assert" $O/pytest_quick.log | head -20; exit $rc; }
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --no-events"
for V in "1 1" "1 0" "0 0" "1 1"; do
  set -- $V
  MGICP_RESIDENT=$1 MGICP_HOST_ROWS=$2 timeout -k 10 300 python -u $B > $O/b_$1$2.json 2> $O/b_$1$2.err || { tail -30 $O/b_$1$2.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$1$2.json')); print('resident $1 rows $2', d['value'], d['ms_per_step'], d['frob_vs_oracle'] if 'frob_vs_oracle' in d else '')"
done

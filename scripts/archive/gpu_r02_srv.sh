# resident pass server: its parity test, C4 bench with the server on / off and its pass times, GPU suite
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/srv; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -k resident -x -v --timeout 240 --timeout-method thread > $O/pytest_resident.log 2>&1
rc=$?; tail -5 $O/pytest_resident.log; [ $rc -ne 0 ] && { grep -n "Error\|assert\|FAIL" $O/pytest_resident.log | head -30; exit $rc; }
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --no-events"
MGICP_PASS_TIMES=1 timeout -k 10 300 python -u $B > $O/b_on.json 2> $O/b_on.err || { tail -30 $O/b_on.err; exit 1; }
grep "pass-times" $O/b_on.err | tail -3
MGICP_RESIDENT=0 timeout -k 10 300 python -u $B > $O/b_off.json 2> $O/b_off.err || { tail -30 $O/b_off.err; exit 1; }
python3 -c "
import json
for n in ('on','off'):
    d=json.load(open('$O/b_'+n+'.json')); print(n, d['value'], d['ms_per_step'], d.get('frob_vs_oracle'), d.get('objective_passes_per_align'))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; exit $rc

# BAR command block + first-sweep seed map: exactness / parity tests, C4 and C2 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/bar; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gicp_gpu.py tests/test_distributed.py tests/test_full_size_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -n "Error\|assert" $O/pytest.log | head; exit $rc; }
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --pass-bench 0 --prof-steps 2"
for V in "1 1" "0 1" "1 0" "1 1"; do
  set -- $V
  MGICP_BAR_CMD=$1 MGICP_SEED_MAP=$2 MGICP_PASS_TIMES=1 timeout -k 10 300 python -u $B > $O/b_C4_$1$2.json 2> $O/b_C4_$1$2.err || { tail -30 $O/b_C4_$1$2.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_C4_$1$2.json')); k=d['kernels']['correspond']; print('C4 bar $1 seedmap $2', d['value'], d['ms_per_step'], 'corr avg ms', round(k['avg_ms'],4), k['count'])"
  grep "host view" $O/b_C4_$1$2.err | tail -1
done
for BAR in 1 0; do
  MGICP_BAR_CMD=$BAR MGICP_PASS_TIMES=1 timeout -k 10 300 python -u $B --config C2 > $O/b_C2_$BAR.json 2> $O/b_C2_$BAR.err || { tail -30 $O/b_C2_$BAR.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_C2_$BAR.json')); print('C2 bar $BAR', d['value'], d['ms_per_step'])"
  grep "host view" $O/b_C2_$BAR.err | tail -1
done

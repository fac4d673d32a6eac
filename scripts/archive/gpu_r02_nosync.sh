# correspondence phase without the host sync: GPU suite, then bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/nosync; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -n "Error\|assert\|FAIL" $O/pytest.log | head; exit $rc; }
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --no-events --pass-bench 0"
for C in C4 C4 C4 C2; do
  timeout -k 10 300 python -u $B --config $C > $O/b_$C.json 2> $O/b_$C.err || { tail -30 $O/b_$C.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$C.json')); print('$C', d['value'], d['ms_per_step'], d.get('gn_mode',{}).get('value'))"
done

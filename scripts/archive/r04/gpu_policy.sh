# r04: 1-NN list build policy -- driver-form C4 bench (--steps 20 --warmup 5) and the second align's wall time
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-policy}; mkdir -p $O
shift
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/b.json 2> $O/b.err || { echo "$cfg bench failed"; tail -5 $O/b.err; exit 1; }
  v=$(python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")
  env $cfg timeout -k 10 300 python3 -u scripts/trace_first_align.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
  a=$(grep -E "^\{" $O/run.log | tail -2 | python3 -c "
import sys, ast
print(' '.join(str(round(ast.literal_eval(l)['ms_total'], 1)) for l in sys.stdin))")
  echo "$cfg: bench it/s, ms/step: $v | new-context align 1, align 2 (ms): $a"
done
echo done

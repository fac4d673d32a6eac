# repeat of the stagger bench A/B (5 runs each, interleaved)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/stagger2; mkdir -p $O
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events --pass-bench 0"
for r in 1 2 3 4 5; do
for L in libmgicp.so libmgicp_stag0.so; do
  MGICP_LIB_NAME=$L timeout -k 10 300 python -u $B > $O/b_${L}_$r.json 2> $O/b_${L}_$r.err || { tail -30 $O/b_${L}_$r.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_${L}_$r.json')); print('$L', d['value'], d['ms_per_step'])"
done
done

# r04: the second align after set_* (the one that builds the 1-NN cell lists): wall time, C4 and C4F, lists on / off
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-align2}; mkdir -p $O
for cfg in "C4F=0" "C4F=1" "C4F=1 MGICP_VLIST=0" "C4F=0 MGICP_VLIST_EAGER=0"; do
  env $cfg timeout -k 10 300 python3 -u scripts/trace_first_align.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
  echo "$cfg: $(grep -E "^\{" $O/run.log | tail -2 | python3 -c "
import sys, ast
for l in sys.stdin: d = ast.literal_eval(l); print(round(d['ms_total'], 1), end=' ms  ')")"
done
echo done

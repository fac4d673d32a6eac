# target grid occupancy A/B with the seeded searches (MGICP_GRID_OCC; default 10)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/occ; mkdir -p $O
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --pass-bench 0 --prof-steps 2"
for OCC in 10 6 8 14 10 6; do
  MGICP_GRID_OCC=$OCC timeout -k 10 300 python -u $B > $O/b_$OCC.json 2> $O/b_$OCC.err || { tail -30 $O/b_$OCC.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$OCC.json')); k=d['kernels']['correspond']; print('occ $OCC', d['value'], d['ms_per_step'], 'corr avg', round(k['avg_ms'],4), 'first', d['ms_to_converge_first'])"
done

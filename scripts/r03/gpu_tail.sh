# r03: the server's timing form with and without its reduction tail (libmgicp_notail.so), C4 and C2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-tail}; mkdir -p $O
for c in C4 C2 C3; do
  for lib in libmgicp.so libmgicp_notail.so; do
    MGICP_LIB_NAME=$lib timeout -k 10 200 python3 bench.py --config $c --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0 > $O/b_${c}_$lib.json 2> $O/b_${c}_$lib.log || { echo "$c $lib failed"; tail -5 $O/b_${c}_$lib.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${c}_$lib.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$c $lib', 'us/pass', round(r['avg_launch_ms']*1e3,2), r['server']['ms_per_pass_runs'])"
  done
done

# r05 A/B: the resident server's cache-warming prefetch before the gate (MGICP_SRV_PREFETCH=2) -- C4 bench lines
# (in-align pass, timing form, C5 pass), alternating default / variant
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-pfab}; mkdir -p $O
B="--cold-pairs 0 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --steps 20"
for rep in 1 2; do
  for v in "" _pf2; do
    MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 300 python3 bench.py $B > $O/b$v.$rep.json 2> $O/b$v.$rep.err || { echo "bench $v failed"; tail -20 $O/b$v.$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b$v.$rep.json')); r=d['roofline']; c5=d['rooflines'].get('fdf_52B_c5_past_infinity_cache') or {}
print('$v rep $rep value', d['value'], 'in-align us', round(r['avg_launch_ms']*1e3,2), 'timing us', round(r['timing_form']['ms_per_pass']*1e3,2), 'c5 us', round(c5.get('avg_launch_ms',0)*1e3,1), 'frob', d['frob_vs_oracle'], 'takeovers', r['pass_stats_timed']['takeovers'])"
  done
done

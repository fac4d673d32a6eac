# bench lines of the other BASELINE.json configs (C2, C3, C5) with the current engine
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
for c in C2 C3 C5; do
  timeout -k 10 400 python bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], 'gn', d['gn_mode']['value'], d['gn_mode']['frob_vs_oracle_gn_sample'], 'frob', d['frob_vs_oracle_sample'], 'cpu', d['cpu_baseline']['value'])"
done
echo done

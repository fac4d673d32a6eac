cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-events}
mkdir -p $OUT
for r in 1 2; do
for v in ev noev; do
  extra=""; [ $v = noev ] && extra="--no-events"
  timeout -k 10 200 python bench.py --steps 20 --warmup 2 --gn-steps 10 --cpu-sample 0 --fod-cpu-sample 0 $extra > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { echo "$v failed"; tail -5 $OUT/${v}_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${v}_$r.json')); print('${v}_$r', d['value'], 'gn', d['gn_mode']['value'])"
done
done

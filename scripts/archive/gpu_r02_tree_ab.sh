# fixed reduction tree: objective-pass grid A/B (persistent 4-wave blocks)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/tree_ab; mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for nb in 256 512 1024 256 512 1024; do MGICP_FDF_BLOCKS=$nb timeout -k 10 200 $B > $O/b$nb.json 2> $O/err$nb || { tail $O/err$nb; exit 1; }
python -c "import json;d=json.load(open('$O/b$nb.json'));print('blocks=$nb',d['value'],d['ms_per_step'],d['kernels']['fdf'])"; done

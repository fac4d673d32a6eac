# logged k-NN kernel: log capacity sweep (per-lane LDS entries), first-align prep
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/knnlog; mkdir -p $O
B="python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for c in 48 32 40 64 96; do MGICP_KNN_STATS=1 MGICP_KNN_LOG=$c timeout -k 10 200 $B > $O/b$c.json 2> $O/err$c || { tail $O/err$c; exit 1; }
 python -c "import json;d=json.load(open('$O/b$c.json'));print('cap=$c',d['kernels']['knn_cov'])"; grep "\[knn\]" $O/err$c | head -2; done
echo done

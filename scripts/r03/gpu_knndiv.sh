# r03: k-NN divergence diagnostic (libmgicp_ph.so: -DMGICP_CORR_PHASES=1 -DMGICP_KNN_DIV=1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-knndiv}; mkdir -p $O
MGICP_LIB_NAME=libmgicp_ph.so timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/b.json 2> $O/b.log || { tail -5 $O/b.log; exit 1; }
grep "knn-div" $O/b.log | sort | uniq -c

# r03: per-phase shader-clock totals of the wave 1-NN sweep (libmgicp_ph.so, MGICP_CORR_PHASES=1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-phase}; mkdir -p $O
shift
for cfg in "$@"; do
  env MGICP_LIB_NAME=libmgicp_ph.so $cfg timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 \
      --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0 --pass-bench 0 > $O/b.json 2> $O/b.log || { echo "failed"; tail -5 $O/b.log; exit 1; }
  echo "== $cfg"; grep "corr-phase" $O/b.log | tail -3
done

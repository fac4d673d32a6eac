# r03: per-pass device active time vs turnaround (MGICP_PASS_TIMES=1), C4 and C2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-passtimes}; mkdir -p $O
for c in C4 C2; do
  MGICP_PASS_TIMES=1 timeout -k 10 200 python3 bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0 --pass-bench 0 > $O/b_$c.json 2> $O/b_$c.log || { echo "$c failed"; tail -5 $O/b_$c.log; exit 1; }
  echo "== $c"; grep "pass-times" $O/b_$c.log | tail -4
done

# r04: the C4F first align's k-NN work (MGICP_KNN_STATS=1): head start, hand-offs, lazy passes per sweep
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-c4fknn}; mkdir -p $O
C4F=1 MGICP_KNN_STATS=1 timeout -k 10 300 python3 -u scripts/trace_first_align.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
grep -E "knn|second context|n_corr" $O/run.log | tail -30
for cap in 6 8; do
  C4F=1 MGICP_KNN_STATS=1 MGICP_ASYNC_RING_CAP=$cap timeout -k 10 300 python3 -u scripts/trace_first_align.py > $O/run_cap$cap.log 2>&1 || { tail -5 $O/run_cap$cap.log; exit 1; }
  echo "cap $cap:"; grep -E "knn|ms_loop" $O/run_cap$cap.log | tail -12
done
echo done

# r06 A/B: grid sizing by the sketch (libmgicp.so) vs the r05 trial histograms (libmgicp_hist.so, the
# previous commit's build), alternating in one box; then the engine GPU tests and a C4 cold-pair trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-sketchab}; mkdir -p $O
for round in 1 2; do
  for lib in libmgicp_hist.so libmgicp.so; do
    for cfg in C4 C4F; do
      MGICP_LIB_NAME=$lib timeout -k 10 200 python scripts/r05/cold_pair.py 4 $cfg > $O/cold_${cfg}_${lib}_$round.txt 2>&1 || { tail -20 $O/cold_${cfg}_${lib}_$round.txt; exit 1; }
      echo "$round $cfg $(tail -1 $O/cold_${cfg}_${lib}_$round.txt)"
    done
  done
done
MGICP_TRACE=1 timeout -k 10 200 python scripts/r05/cold_pair.py 1 > $O/cold_c4_trace.txt 2> $O/trace_c4.txt || { echo "trace failed"; tail -20 $O/trace_c4.txt; exit 1; }
grep "grid" $O/trace_c4.txt | head -20
timeout -k 10 700 python -u -m pytest tests/test_gicp_gpu.py tests/test_parity_configs_gpu.py -m gpu -x -v -k "not C5 and not C3" --timeout 300 --timeout-method thread > $O/pytest_gicp.log 2>&1 || { tail -30 $O/pytest_gicp.log; exit 1; }
tail -2 $O/pytest_gicp.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/C4 -o run -- python3 scripts/r05/cold_pair.py 1 > $O/coldprof_C4.txt 2>&1 || { tail -5 $O/coldprof_C4.txt; exit 1; }
echo done

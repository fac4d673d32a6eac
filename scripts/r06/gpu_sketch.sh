# r06: the sketch-sized grid (no trial histograms): grid sizes chosen, cold-pair timings, the GPU
# suite's engine tests, and a kernel trace of the C4 cold pair
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-sketch}; mkdir -p $O
MGICP_TRACE=1 timeout -k 10 200 python scripts/r05/cold_pair.py 1 > $O/cold_c4_trace.txt 2> $O/trace_c4.txt || { echo "trace failed"; tail -20 $O/trace_c4.txt; exit 1; }
grep "grid" $O/trace_c4.txt | head -20
timeout -k 10 200 python scripts/r05/cold_pair.py 3 > $O/cold_c4.txt 2>&1 || { tail -20 $O/cold_c4.txt; exit 1; }
cat $O/cold_c4.txt
timeout -k 10 200 python scripts/r05/cold_pair.py 3 C4F > $O/cold_c4f.txt 2>&1 || { tail -20 $O/cold_c4f.txt; exit 1; }
cat $O/cold_c4f.txt
timeout -k 10 700 python -u -m pytest tests/test_gicp_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gicp.log 2>&1 || { tail -30 $O/pytest_gicp.log; exit 1; }
tail -3 $O/pytest_gicp.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/C4 -o run -- python3 scripts/r05/cold_pair.py 1 > $O/coldprof_C4.txt 2>&1 || { tail -5 $O/coldprof_C4.txt; exit 1; }
echo done

# r06 A/B of two builds (cold pairs at C4 / C4F, alternating, two rounds), then the engine + parity GPU
# tests and a kernel trace of one C4 cold pair on libmgicp.so.  usage: gpu_ab.sh OUT LIB_A LIB_B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-ab}; mkdir -p $O
A=${2:-libmgicp_prev.so}; B=${3:-libmgicp.so}
for round in 1 2; do
  for lib in $A $B; do
    for cfg in C4 C4F; do
      MGICP_LIB_NAME=$lib timeout -k 10 200 python scripts/r05/cold_pair.py 4 $cfg > $O/cold_${cfg}_${lib}_$round.txt 2>&1 || { tail -20 $O/cold_${cfg}_${lib}_$round.txt; exit 1; }
      echo "$round $cfg $(tail -1 $O/cold_${cfg}_${lib}_$round.txt)"
    done
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gicp_gpu.py tests/test_parity_configs_gpu.py -m gpu -x -v -k "not C5 and not C3" --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|Timeout" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/C4 -o run -- python3 scripts/r05/cold_pair.py 1 > $O/coldprof_C4.txt 2>&1 || { tail -5 $O/coldprof_C4.txt; exit 1; }
echo done

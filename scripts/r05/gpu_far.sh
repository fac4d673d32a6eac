# r05: far-straggler hand-off in the cold 1-NN sweep -- its bit-exactness test + the sweep/parity tests, then
# C4F and C4 GICPState cycles with the hand-off off (default) and on
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-far}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gicp_gpu.py tests/test_full_size_gpu.py tests/test_parity_configs_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu -k "far or vlist or c4f or C4F or C2F or C4 or brute or fused or lazy" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in C4F C4; do
  timeout -k 10 200 python scripts/r05/cold_pair.py 3 $w > $O/cold_$w.txt 2>&1 || { echo "cold $w failed"; tail -20 $O/cold_$w.txt; exit 1; }
  echo "$w off: $(tail -1 $O/cold_$w.txt)"
  MGICP_COLD_OPTS=corr_far_split=1 timeout -k 10 200 python scripts/r05/cold_pair.py 3 $w > $O/cold_${w}_off.txt 2>&1 || { echo "cold $w off failed"; tail -20 $O/cold_${w}_off.txt; exit 1; }
  echo "$w on: $(tail -1 $O/cold_${w}_off.txt)"
done

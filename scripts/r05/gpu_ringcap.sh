# r05 A/B: rings the lazy source's head-start k-NN searches (MGICP_ASYNC_RING_CAP 1/2/3 vs 4) -- C4F and C4 GICPState
# cycles (cold_pair.py: cycle 1 cold, then the target cache)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-ringcap}; mkdir -p $O
for w in C4F C4; do
  for v in "" _rc3 _rc2 _rc1; do
    MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 200 python scripts/r05/cold_pair.py 3 $w > $O/cold_$w$v.txt 2>&1 || { echo "cold $w $v failed"; tail -20 $O/cold_$w$v.txt; exit 1; }
    echo "$w cap${v:-4}: $(tail -1 $O/cold_$w$v.txt)"
  done
done

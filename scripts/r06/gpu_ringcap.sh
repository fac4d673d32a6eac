# r06: the source head start's ring cap with the wave-per-query lazy pass -- cold pairs at C4 / C4F
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-ringcap}; mkdir -p $O
for cap in 4 2 1 3; do
  for cfg in C4F C4; do
    MGICP_COLD_OPTS="async_ring_cap=$cap" timeout -k 10 200 python scripts/r05/cold_pair.py 3 $cfg > $O/cold_${cfg}_cap$cap.txt 2>&1 || { tail -5 $O/cold_${cfg}_cap$cap.txt; exit 1; }
    echo "cap $cap $cfg: $(tail -1 $O/cold_${cfg}_cap$cap.txt)"
  done
done

# r04 A/B of the new-clouds path: new_clouds_trace.py (both set_* orders) under several env settings
# usage: gpu_ncab.sh OUTNAME "ENV1" "ENV2" ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-ncab}; mkdir -p $O
shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  for sf in 0 1; do
    env $cfg SOURCE_FIRST=$sf timeout -k 10 300 python3 -u scripts/r04/new_clouds_trace.py > $O/c${i}_sf$sf.txt 2> $O/c${i}_sf$sf.err || { echo "$cfg failed"; tail -5 $O/c${i}_sf$sf.err; exit 1; }
    echo "$cfg sf=$sf: $(awk '{for(i=1;i<=NF;i++) if($i=="total") print $(i+1)}' $O/c${i}_sf$sf.txt | tr '\n' ' ')"
  done
done
echo done

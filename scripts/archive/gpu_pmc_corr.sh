# SQ counters of the 1-NN kernels (tiled and global) on a short C4 bench, separate passes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_corr}
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for tc in 1 0; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    MGICP_TILE_CORR=$tc timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/tc${tc}_p$i -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 > $OUT/tc${tc}_p$i.log 2>&1 || { echo "pmc tc$tc p$i failed"; tail -5 $OUT/tc${tc}_p$i.log; exit 1; }
    python3 scripts/pmc_kernels.py $OUT/tc${tc}_p$i correspond > $OUT/tc${tc}_p$i.txt
    cat $OUT/tc${tc}_p$i.txt
    find $OUT/tc${tc}_p$i -name "*.csv" -size +5M -delete
  done
done
echo done

# r03: SQ + TA counters of one kernel family over a short C4 bench (args: out-name kernel-substring)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/$1; K=$2; mkdir -p $O
B="bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU --output-format csv -d $O/p1 -o run -- python3 $B > $O/p1.log 2>&1 || { echo "p1 failed"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d $O/p2 -o run -- python3 $B > $O/p2.log 2>&1 || { echo "p2 failed"; tail -20 $O/p2.log; exit 1; }
python3 scripts/r03/pmc_dispatch.py $O/p1 $K | head -3
python3 scripts/r03/pmc_dispatch.py $O/p2 $K | head -3
find $O -name "*.csv" -size +20M -delete
echo done

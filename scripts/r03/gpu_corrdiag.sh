# r03: where the 1-NN sweep's time goes at C4 -- per-sweep work counts (MGICP_CORR_STATS build),
# per-dispatch durations (kernel trace) and SQ counters (one PMC pass), sweeps in launch order
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/corrdiag; mkdir -p $O
B="bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0"
MGICP_LIB_NAME=libmgicp_stats.so timeout -k 10 300 python3 $B > $O/stats.json 2> $O/stats.log || { tail -20 $O/stats.log; exit 1; }
grep corr-stats $O/stats.log | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $B > $O/kt.json 2> $O/kt.log || { tail -20 $O/kt.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU --output-format csv -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 || { echo "sq failed"; tail -20 $O/sq.log; exit 1; }
python3 scripts/r03/per_dispatch.py $O correspond_kernel compact_kernel
find $O -name "*.csv" -size +20M -delete
echo done

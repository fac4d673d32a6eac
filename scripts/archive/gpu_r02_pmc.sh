# round-2 PMC passes (each counter group in its own run, no trace domains): HBM bytes per kernel
# (FETCH_SIZE, WRITE_SIZE) and SQ instruction mix; C4 bench without the CPU legs
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/pmc; mkdir -p $O
B="bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --prof-steps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1 || { echo "write failed"; tail -20 $O/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU --output-format csv -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 || { echo "sq failed"; tail -20 $O/sq.log; exit 1; }
python3 scripts/pmc_summary.py $O/fetch $O/write 5000000 1 $O/pmc_summary.json > /dev/null && echo summary ok
python3 scripts/pmc_kernels.py $O/sq > $O/sq_summary.txt 2>&1; head -60 $O/sq_summary.txt
find $O -name "*.csv" -size +20M -delete
echo done

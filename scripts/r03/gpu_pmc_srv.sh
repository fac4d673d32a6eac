# r03: SQ counters of the resident server's timing form (fdf_server_kernel<true, 4>) and the sweeps
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-pmcsrv}; mkdir -p $O
B="bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0 --pass-bench 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/sq1 -o run -- python3 $B > $O/sq1.log 2>&1 || { echo "sq1 failed"; tail -5 $O/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/sq2 -o run -- python3 $B > $O/sq2.log 2>&1 || { echo "sq2 failed"; tail -5 $O/sq2.log; exit 1; }
python3 scripts/pmc_kernels.py $O/sq1 fdf_server correspond > $O/sq1.txt 2>&1; cat $O/sq1.txt
python3 scripts/pmc_kernels.py $O/sq2 fdf_server correspond > $O/sq2.txt 2>&1; cat $O/sq2.txt
find $O -name "*.csv" -delete
echo done

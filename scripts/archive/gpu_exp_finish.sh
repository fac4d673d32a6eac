# regression tests, then A/B of the sc1 in-launch finish at several grid sizes + SQ counters
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_5.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_5.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_5.log
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab3_$name.json 2> gpurun_out/ab3_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/ab3_$name.err; exit 1; }; }
run b256 MGICP_FDF_BLOCKS=256
run b512 MGICP_FDF_BLOCKS=512
run b1024 MGICP_FDF_BLOCKS=1024
run b2048 MGICP_FDF_BLOCKS=2048
run b128 MGICP_FDF_BLOCKS=128
run sep512 MGICP_FDF_BLOCKS=512 MGICP_FUSED_FINISH=0
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -20 gpurun_out/pmc_sq.log; exit 1; }
echo done

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/knn2pmc; mkdir -p $O
B="bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 1"
for v in 1; do
MGICP_KNN2=$v timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/sq$v -o run -- python3 $B > $O/sq$v.log 2>&1 || { echo "sq failed"; tail -20 $O/sq$v.log; exit 1; }
python3 scripts/pmc_kernels.py $O/sq$v knn_cov
done
find $O -name "*.csv" -size +20M -delete

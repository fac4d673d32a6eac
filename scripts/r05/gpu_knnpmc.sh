# r05: SQ counters of the k-NN covariance kernels (knn_time.py under rocprofv3 --pmc), per library variant
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05/knnpmc}
shift
mkdir -p $O
for v in "$@"; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $O/sq$v -o run -- python3 scripts/r05/knn_time.py > $O/sq$v.log 2>&1 || { echo "sq $v failed"; tail -20 $O/sq$v.log; exit 1; }
  python3 scripts/pmc_kernels.py $O/sq$v knn_ > $O/sq_summary$v.txt 2>&1
  cat $O/sq_summary$v.txt
done

# r05: cold-pair timing per library variant, then a rocprofv3 kernel trace of the default one
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05/cold}
shift
mkdir -p $OUT
for v in "$@"; do
  MGICP_LIB_NAME=libmgicp$v.so timeout -k 10 200 python scripts/r05/cold_pair.py 4 > $OUT/cold$v.txt 2>&1 || { echo "cold $v failed"; tail -20 $OUT/cold$v.txt; exit 1; }
  tail -1 $OUT/cold$v.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 scripts/r05/cold_pair.py 3 > $OUT/cold_prof.txt 2>&1 || { echo "prof failed"; tail -20 $OUT/cold_prof.txt; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-8

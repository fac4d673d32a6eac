# r05 diagnostics: k-NN time vs grid occupancy; correspondence-sweep phases of the cold pair (MGICP_CORR_PHASES build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-diag}; mkdir -p $O
timeout -k 10 300 python scripts/r05/knn_occ.py 4 6 8 10 14 20 > $O/knn_occ.txt 2>&1 || { echo "knn_occ failed"; tail -20 $O/knn_occ.txt; exit 1; }
cat $O/knn_occ.txt
MGICP_LIB_NAME=libmgicp_cph.so timeout -k 10 200 python scripts/r05/cold_pair.py 2 > $O/cph.txt 2> $O/cph_err.txt || { echo "cph failed"; tail -20 $O/cph_err.txt; exit 1; }
grep "corr-phase" $O/cph_err.txt | tail -6
MGICP_LIB_NAME=libmgicp_kdiv.so timeout -k 10 200 python scripts/r05/knn_time.py > $O/kdiv.txt 2>&1 || { echo "kdiv failed"; tail -20 $O/kdiv.txt; exit 1; }
grep -E "knn-div|knn_cov per" $O/kdiv.txt | tail -3

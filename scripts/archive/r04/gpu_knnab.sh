# r04 A/B: k-NN covariance time per 5M cloud (scripts/r04/knn_time.py) under variant builds / env
# usage: gpu_knnab.sh OUTNAME "ENV1" "ENV2" ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-knnab}; mkdir -p $O
shift
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gicp_gpu.py -k "covariances_bitexact or logged_knn" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python3 -u scripts/r04/knn_time.py >> $O/knn.txt 2> $O/knn.err || { echo "$cfg failed"; tail -5 $O/knn.err; exit 1; }
    echo "$cfg: $(tail -1 $O/knn.txt)"
  done
done
echo done

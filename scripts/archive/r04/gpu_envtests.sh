# r04: one pytest -k selection under several env settings (diagnosis), e.g.
# gpu_envtests.sh OUT "detached_shards" "MGICP_ASYNC_COV=0" "MGICP_LAZY_SRC_COV=0"
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-envtests}; mkdir -p $O
K=$2
shift 2
i=0
for cfg in "X=0" "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "$K" > $O/t$i.log 2>&1
  rc=$?
  echo "$cfg: rc=$rc $(tail -1 $O/t$i.log)"
  [ $rc -gt 1 ] && [ $rc -ne 5 ] && { echo "stopping: rc $rc"; exit 1; }
done
echo done

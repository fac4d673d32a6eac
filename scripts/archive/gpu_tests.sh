# GPU parity suite only (fast iteration): pytest -m gpu [extra pytest args]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tests}
shift || true
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu "$@" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log

# r04: a selection of GPU tests (-k EXPR), then C4 and C4F bench lines and the new-clouds breakdown
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-quick3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "$2" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in C4 C4F; do
  timeout -k 10 400 python3 -u bench.py --config $c --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -30 $O/bench_$c.err; exit 1; }
  python3 scripts/r04/show_bench.py $O/bench_$c.json
done
bash scripts/r04/gpu_newclouds.sh ${1:-quick3}_nc

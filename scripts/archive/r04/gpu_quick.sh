# r04: a selection of GPU tests (-k EXPR), the C4 bench line and the new-clouds kernel timeline
# usage: gpu_quick.sh OUTNAME "pytest -k expression"
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-quick}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "$2" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/bench_C4.json 2> $O/bench_C4.err || { echo "bench failed"; tail -30 $O/bench_C4.err; exit 1; }
python3 scripts/r04/show_bench.py $O/bench_C4.json
bash scripts/r04/gpu_prep.sh ${1:-quick}_prep > /dev/null && head -3 gpurun_out/r04/${1:-quick}_prep/timeline.txt
echo done

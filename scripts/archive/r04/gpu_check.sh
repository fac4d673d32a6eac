# r04: verify the tree on the GPU -- suite, smoke, C4 and C4F bench lines (+ rocprof kernel stats of C4F)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-check}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -rP > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
grep -E "^C[0-9]F?:" $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench_C4.json 2> $O/bench_C4.err || { echo "bench failed"; tail -30 $O/bench_C4.err; exit 1; }
python3 scripts/r04/show_bench.py $O/bench_C4.json
timeout -k 10 400 python3 -u bench.py --config C4F --gn-steps 0 > $O/bench_C4F.json 2> $O/bench_C4F.err || { echo "bench C4F failed"; tail -30 $O/bench_C4F.err; exit 1; }
python3 scripts/r04/show_bench.py $O/bench_C4F.json
echo done

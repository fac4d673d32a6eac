# r06 check: GPU suite, smoke, default C4 and C4F bench lines -> gpurun_out/r06/<name>
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-check}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -rP > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench_C4.json 2> $O/bench_C4.err || { tail -30 $O/bench_C4.err; exit 1; }
python3 scripts/r05/show_bench.py $O/bench_C4.json
timeout -k 10 120 python3 scripts/r06/dump_order.py C4F $O/order_C4F.npy && timeout -k 10 400 python3 -u bench.py --config C4F --gn-steps 0 --cold-pairs 1 --c5-leg 0 > $O/bench_C4F.json 2> $O/bench_C4F.err || { tail -30 $O/bench_C4F.err; exit 1; }
python3 scripts/r05/show_bench.py $O/bench_C4F.json
echo done

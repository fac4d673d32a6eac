# A/B: per-cell point boxes in the 1-NN sweeps (MGICP_CELL_BOXES), exactness tests, work counters,
# and a kernel trace of the C4 bench for the host-turnaround gaps
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/boxes; mkdir -p $O
B="python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 5"
timeout -k 10 300 python -u -m pytest tests/test_gicp_gpu.py tests/test_full_size_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0 1 0; do MGICP_CELL_BOXES=$v timeout -k 10 200 $B > $O/bench_boxes$v.json 2>$O/err || { tail $O/err; exit 1; }; python -c "import json;d=json.load(open('$O/bench_boxes$v.json'));print('boxes=$v',d['value'],d['kernels']['correspond'],d['gn_mode']['value'],d['ms_to_converge_first_detail'])"; done
MGICP_LIB_NAME=libmgicp_stats.so MGICP_CELL_BOXES=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/stats1.json 2> $O/stats1.err; grep corr-stats $O/stats1.err | head -6
MGICP_LIB_NAME=libmgicp_stats.so MGICP_CELL_BOXES=0 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/stats0.json 2> $O/stats0.err; grep corr-stats $O/stats0.err | head -6
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/kt_bench.json 2> $O/kt.err || { tail $O/kt.err; exit 1; }
find $O/kt -name "*kernel_trace.csv" | head -2
echo done

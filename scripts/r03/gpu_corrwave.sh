# r03: wave-uniform 1-NN sweep -- exactness tests, per-sweep work counts, timing vs the per-lane kernel
# and over the union / per-lane switch (MGICP_CORR_UNION_MIN_R)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-corrwave}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gicp_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0"
MGICP_LIB_NAME=libmgicp_stats.so timeout -k 10 300 python3 $B --steps 1 --warmup 1 > $O/stats.json 2> $O/stats.log || { tail -20 $O/stats.log; exit 1; }
grep corr-stats $O/stats.log | head -3
for cfg in "MGICP_CORR_WAVE=0" "MGICP_CORR_UNION_MIN_R=0" "MGICP_CORR_UNION_MIN_R=0.5" "MGICP_CORR_UNION_MIN_R=1" ${EXTRA_CFGS}; do
  env $cfg timeout -k 10 300 python3 $B > $O/bench_$cfg.json 2> $O/bench_$cfg.log || { tail -20 $O/bench_$cfg.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$cfg.json'));print('$cfg', d['value'], 'it/s', d['ms_per_step'], 'ms')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $B --steps 1 --warmup 1 > $O/kt.json 2> $O/kt.log || { tail -20 $O/kt.log; exit 1; }
python3 scripts/r03/per_dispatch.py $O correspond_wave_kernel correspond_kernel
find $O -name "*.csv" -size +20M -delete
echo done

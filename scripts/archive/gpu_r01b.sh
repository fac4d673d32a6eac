# r01 (session 5) GPU pass: gpu tests, smoke, C4 bench (BFGS + GN + FOD rows + CPU baselines),
# kernel-trace stats of the same bench, FETCH_SIZE / WRITE_SIZE in their own --pmc passes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r01b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench_C4.json 2> $OUT/bench_C4.err || { echo "bench failed"; tail -20 $OUT/bench_C4.err; exit 1; }
echo bench ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/bench_under_kt.json 2> $OUT/kt.err || { echo "kernel trace failed"; tail -20 $OUT/kt.err; exit 1; }
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --gn-steps 2 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --gn-steps 2 --cpu-sample 0 --fod-cpu-sample 0 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
python3 scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write fdf_soa_kernel 5000000 1 $OUT/r01_pmc_fdf.json
find $OUT/kt $OUT/pmc_fetch $OUT/pmc_write -name "*.csv" -size +5M -delete
echo done

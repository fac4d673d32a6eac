# round-1 profiles of the final engine at C4: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE
# in their own --pmc passes (no trace domains combined with counters)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/kt -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof/bench_under_kt.json 2> gpurun_out/prof/kt.err || { echo "kernel trace failed"; tail -20 gpurun_out/prof/kt.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/prof/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/prof/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/prof/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/prof/pmc_write.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof/pmc_fetch gpurun_out/prof/pmc_write fdf_soa_kernel 5000000 1 gpurun_out/prof/r01_pmc_fdf.json
# keep only the summaries (counter CSVs are large)
find gpurun_out/prof/pmc_fetch gpurun_out/prof/pmc_write -name "*.csv" -size +20M -delete
echo done

# PMC passes (separate from any trace domain): FETCH_SIZE and WRITE_SIZE of the objective pass
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write fdf_soa_kernel 5000000 1 gpurun_out/r01_pmc_fdf.json
ls -R gpurun_out/pmc_fetch | head
echo done

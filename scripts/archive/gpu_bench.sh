set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
nproc > gpurun_out/host_nproc.txt; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Core" >> gpurun_out/host_nproc.txt
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-sample 200000 > gpurun_out/bench_r01_a.json 2> gpurun_out/bench_r01_a.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r01 -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bench_r01_prof.json 2> gpurun_out/bench_r01_prof.err
echo done

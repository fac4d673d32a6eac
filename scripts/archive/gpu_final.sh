# Round-end evidence for HEAD: default bench line + rocprofv3 kernel-trace stats of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_C4_final2.json 2> gpurun_out/bench_C4_final2.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_final2 -o run -- python bench.py --cpu-sample 0 --fod-cpu-sample 0 > gpurun_out/bench_C4_final2_prof.json 2> gpurun_out/bench_C4_final2_prof.err || exit 1
echo done

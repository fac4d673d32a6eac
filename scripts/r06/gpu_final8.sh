# r06 check8: list-build timings (vlb_time.py, both libraries), the full GPU suite + smoke + C4 / C4F bench lines
# (gpu_check.sh), then rocprofv3 kernel stats of the C4 bench command -> gpurun_out/r06/{vlb5,check8,prof8}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/r06/gpu_vlb.sh vlb5 || exit 1
bash scripts/r06/gpu_check.sh check8 || exit 1
O=gpurun_out/r06/prof8; mkdir -p $O
B="bench.py --steps 3 --warmup 5 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --cold-pairs 1 --c5-leg 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -o run -- python3 $B > $O/b_c4_under_rocprof.json 2> $O/kt_c4.log || { tail -20 $O/kt_c4.log; exit 1; }
f=$(find $O/kt_c4 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_bench_c4.csv
find $O -name "*kernel_trace.csv" -delete
echo done

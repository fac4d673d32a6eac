# r06 evidence, part B: rocprofv3 kernel-trace stats of the C4 / C4F / C3 bench commands and PMC passes
# (each counter group in its own run, no trace domains) -> gpurun_out/r06/<name>
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-final}; mkdir -p $O
B="bench.py --steps 3 --warmup 5 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --cold-pairs 1 --c5-leg 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -o run -- python3 $B > $O/b_c4_under_rocprof.json 2> $O/kt_c4.log || { tail -20 $O/kt_c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4f -o run -- python3 $B --config C4F > $O/b_c4f_under_rocprof.json 2> $O/kt_c4f.log || { tail -20 $O/kt_c4f.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o run -- python3 $B --config C3 > $O/b_c3_under_rocprof.json 2> $O/kt_c3.log || { tail -20 $O/kt_c3.log; exit 1; }
P="bench.py --steps 2 --warmup 5 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --prof-steps 1 --cold-pairs 0 --c5-leg 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $P > $O/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $P > $O/write.log 2>&1 || { echo "write failed"; tail -20 $O/write.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU --output-format csv -d $O/sq -o run -- python3 $P > $O/sq.log 2>&1 || { echo "sq failed"; tail -20 $O/sq.log; exit 1; }
PASS_BENCH_PASSES=50 python3 scripts/pmc_summary.py $O/fetch $O/write 5000000 1 $O/pmc_summary.json > /dev/null && echo summary ok
python3 scripts/pmc_kernels.py $O/sq > $O/sq_summary.txt 2>&1
for d in kt_c4 kt_c4f kt_c3; do f=$(find $O/$d -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats_bench_${d#kt_}.csv; done
find $O -name "*.csv" -size +20M -delete
find $O -name "*kernel_trace.csv" -delete
echo done

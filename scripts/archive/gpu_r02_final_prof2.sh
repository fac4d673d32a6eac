# round-2 measurement evidence (resident pass server + host rows): rocprofv3 kernel-trace stats of the C4 and C3 bench commands, then
# the PMC passes (each counter group in its own run, no trace domains; gated passes off so every
# dispatch completes on its own) for HBM bytes per launch
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/final2; mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench_C4_default.json 2> $O/bench_C4_default.err || { tail -30 $O/bench_C4_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_C4_default.json')); r=d['roofline']
print('bench', d['value'], d['ms_per_step'], 'frac', r['frac'], 'ms/pass', r['avg_launch_ms'], 'launched', d['rooflines']['fdf_launched_52B']['avg_launch_ms'])"
B="bench.py --steps 3 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -o run -- python3 $B > $O/b_c4.json 2> $O/kt_c4.log || { tail -20 $O/kt_c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o run -- python3 $B --config C3 > $O/b_c3.json 2> $O/kt_c3.log || { tail -20 $O/kt_c3.log; exit 1; }
P="bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 2 --prof-steps 1"
export MGICP_GATED=0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $P > $O/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $P > $O/write.log 2>&1 || { echo "write failed"; tail -20 $O/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU --output-format csv -d $O/sq -o run -- python3 $P > $O/sq.log 2>&1 || { echo "sq failed"; tail -20 $O/sq.log; exit 1; }
PASS_BENCH_PASSES=50 python3 scripts/pmc_summary.py $O/fetch $O/write 5000000 1 $O/pmc_summary.json > /dev/null && echo summary ok
python3 scripts/pmc_kernels.py $O/sq > $O/sq_summary.txt 2>&1
find $O -name "*.csv" -size +20M -delete
find $O -name "*kernel_trace.csv" -delete
echo done

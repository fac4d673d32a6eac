# r06 list-build A/B: the vlist tests on the new build, then vlb_time.py on both libraries, then a kernel
# trace of the new one.  usage: gpu_vlb.sh OUT [LIB_A] [LIB_B]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-vlb}; mkdir -p $O
A=${2:-libmgicp_prev.so}; B=${3:-libmgicp.so}
timeout -k 10 600 python -u -m pytest tests/test_gicp_gpu.py -m gpu -x -v -k "vlist or fused_compaction" --timeout 300 --timeout-method thread > $O/pytest_vlist.log 2>&1 || { grep -E "FAILED|Error|Timeout" $O/pytest_vlist.log | head; tail -5 $O/pytest_vlist.log; exit 1; }
tail -1 $O/pytest_vlist.log
for lib in $A $B; do
  MGICP_LIB_NAME=$lib timeout -k 10 300 python3 -u scripts/r06/vlb_time.py $VLB_ARGS > $O/vlb_${lib}.txt 2>&1 || { tail -20 $O/vlb_${lib}.txt; exit 1; }
  grep -v '^SUMMARY' $O/vlb_${lib}.txt | sed "s/^/$lib /"
  grep '^SUMMARY' $O/vlb_${lib}.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/r06/vlb_time.py > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O/kt -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
python3 - $O/kernel_stats.csv <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f"{r['Name'][:48]:48s} calls {r['Calls']:>6s} total {float(r['TotalDurationNs'])/1e6:9.2f} ms avg {float(r['AverageNs'])/1e3:9.1f} us")
EOF
echo done

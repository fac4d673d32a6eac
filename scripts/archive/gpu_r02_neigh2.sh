# seeded sweeps also testing the seed map's candidate: correspondence kernel times (per sweep) A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/neigh2; mkdir -p $O
MGICP_LIB_NAME=libmgicp_neigh2.so timeout -k 10 400 python -u -m pytest tests/test_gicp_gpu.py tests/test_full_size_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -n "Error\|assert" $O/pytest.log | head; exit $rc; }
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --pass-bench 0 --prof-steps 3"
for L in libmgicp.so libmgicp_neigh2.so libmgicp.so libmgicp_neigh2.so; do
  MGICP_LIB_NAME=$L timeout -k 10 300 python -u $B > $O/b_$L.json 2> $O/b_$L.err || { tail -30 $O/b_$L.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_$L.json')); k=d['kernels']['correspond']; print('$L', d['value'], d['ms_per_step'], 'corr avg', round(k['avg_ms'],4))"
done
MGICP_LIB_NAME=libmgicp_neigh2.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --pass-bench 0 --no-events > $O/kt.json 2> $O/kt.log || { tail -5 $O/kt.log; exit 1; }
python3 - <<'PY'
import csv,glob
rows=[r for r in csv.DictReader(open(glob.glob('gpurun_out/r02/neigh2/kt/**/*kernel_trace.csv',recursive=True)[0])) if 'correspond_kernel' in r['Kernel_Name']]
print('per-sweep us:', [round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3,1) for r in rows])
PY
timeout -k 10 400 python -u -m pytest tests/test_distributed.py -m gpu -k "server_forms or resident" -x -q --timeout 300 --timeout-method thread > $O/pytest_forms.log 2>&1
rc=$?; tail -1 $O/pytest_forms.log; exit $rc

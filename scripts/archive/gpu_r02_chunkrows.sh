# per-chunk host rows for small shards: parity tests and C2 / C3 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/chunkrows; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_distributed.py tests/test_parity_configs_gpu.py tests/test_gicp_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -n "Error\|assert" $O/pytest.log | head; exit $rc; }
B="bench.py --steps 10 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events --pass-bench 0"
for CR in 256 0 256 0; do
  MGICP_CHUNK_ROWS=$CR MGICP_PASS_TIMES=1 timeout -k 10 300 python -u $B --config C2 > $O/b_C2_$CR.json 2> $O/b_C2_$CR.err || { tail -30 $O/b_C2_$CR.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_C2_$CR.json')); print('C2 chunk_rows_max $CR', d['value'], d['ms_per_step'])"
  grep "host view" $O/b_C2_$CR.err | tail -2 | head -1
done
for CR in 1024 0; do
  MGICP_CHUNK_ROWS=$CR timeout -k 10 300 python -u $B --config C3 > $O/b_C3_$CR.json 2> $O/b_C3_$CR.err || { tail -30 $O/b_C3_$CR.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/b_C3_$CR.json')); print('C3 chunk_rows_max $CR', d['value'], d['ms_per_step'])"
done

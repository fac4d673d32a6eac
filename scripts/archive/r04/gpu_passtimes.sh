# r04: per-pass timing diagnostics of the resident server in the aligns (MGICP_PASS_TIMES=1, MGICP_GATE_TRACE=1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-passtimes}; mkdir -p $O
B="bench.py --steps 5 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --pass-bench 0"
MGICP_PASS_TIMES=1 timeout -k 10 300 python3 -u $B > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
grep -E "pass-times" $O/b.err | tail -6
python3 scripts/r04/show_bench.py $O/b.json
echo done

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/gtrace; mkdir -p $O
MGICP_GATE_TRACE=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
grep gate-trace $O/b.err | tail -4
MGICP_GATE_TRACE=1 timeout -k 10 200 python -u bench.py --config C2 --steps 3 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events > $O/b2.json 2> $O/b2.err || { tail $O/b2.err; exit 1; }
grep gate-trace $O/b2.err | tail -3

# host-side phase trace of the first align (upload, grid builds, covariances)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MGICP_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/trace_prep.json 2> gpurun_out/trace_prep.err || { echo "bench failed"; tail -5 gpurun_out/trace_prep.err; exit 1; }
grep mgicp gpurun_out/trace_prep.err | head -20

# round 2: GPU suite (incl. full-size C2/C3/C4 oracle parity, adapter replay) then the default bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
echo "host: $(nproc) cpus, OMP_NUM_THREADS=$OMP_NUM_THREADS"; lscpu | grep -i "model name"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r02/pytest_gpu.log
[ $rc -ne 0 ] && { grep -n "FAIL\|Error\|error" gpurun_out/r02/pytest_gpu.log | head -40; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/r02/bench_C4.json 2> gpurun_out/r02/bench_C4.err || { tail -30 gpurun_out/r02/bench_C4.err; exit 1; }
cat gpurun_out/r02/bench_C4.json | head -c 1500
echo
echo done

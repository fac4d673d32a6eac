# gated (pre-launched) objective passes: correctness suite, then A/B bench gated vs plain
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/gated; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gicp_gpu.py tests/test_gicp_alignment.py tests/test_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="python -u bench.py --steps 20 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0"
for v in 1 0 1 0; do MGICP_GATED=$v timeout -k 10 200 $B > $O/bench_g$v.json 2>$O/err || { tail $O/err; exit 1; }; python -c "import json;d=json.load(open('$O/bench_g$v.json'));print('gated=$v',d['value'],d['ms_per_step'],d['kernels']['fdf'])"; done
for c in C2 C3; do for v in 1 0; do MGICP_GATED=$v timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 > $O/bench_${c}_g$v.json 2>$O/err || { tail $O/err; exit 1; }; python -c "import json;d=json.load(open('$O/bench_${c}_g$v.json'));print('$c gated=$v',d['value'],d['ms_per_step'])"; done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events > $O/kt_bench.json 2> $O/kt.err || { tail $O/kt.err; exit 1; }
echo done

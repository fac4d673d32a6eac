# r06: rocprofv3 kernel trace of the cold pair (C4F then C4), one repeat each
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-coldprof}; mkdir -p $O
for cfg in C4F C4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/$cfg -o run -- python3 scripts/r05/cold_pair.py 1 $cfg > $O/cold_$cfg.txt 2>&1 || { tail -5 $O/cold_$cfg.txt; exit 1; }
done
ls -R $O | head

# r04: host-side phase stamps (MGICP_TRACE=1) of the second align after set_* (C4)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-align2trace}; mkdir -p $O
MGICP_TRACE=1 timeout -k 10 300 python3 -u scripts/trace_first_align.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
awk '/second context/{f=1} f' $O/run.log | grep -n "" | tail -80

# objective pass of the fixed reduction tree: where the time goes (diagnostic variants x grid sizes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export MGICP_PROF_STRIDE=1 PYTHONPATH=$GRAFT_REPO_ROOT
for nb in 512; do for d in 0 4 0; do
 echo -n "blocks=$nb diag=$d "; MGICP_FDF_BLOCKS=$nb MGICP_FDF_DIAG=$d timeout -k 10 120 python -u scripts/fdf_timing.py || exit 1
done; done

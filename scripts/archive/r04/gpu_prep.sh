# r04: kernel timeline of a warm-process first align (new clouds): where ms_prep goes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-prep}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 scripts/trace_first_align.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 scripts/r04/prep_timeline.py $O/kt | tee $O/timeline.txt
find $O -name "*.csv" -delete

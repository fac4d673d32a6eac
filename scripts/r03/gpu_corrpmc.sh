# r03: memory-pipe counters of the 1-NN sweeps (is the vector-memory address path the limit?)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03/corrpmc; mkdir -p $O
B="bench.py --steps 1 --warmup 1 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --prof-steps 0"
timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_TCP_TA_DATA_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $B > $O/p1.log 2>&1 || { echo "p1 failed"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TA_FLAT_READ_WAVEFRONTS TA_TOTAL_WAVEFRONTS TD_LOAD_WAVEFRONT TD_COALESCABLE_WAVEFRONT TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_TOTAL_READ GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $B > $O/p2.log 2>&1 || { echo "p2 failed"; tail -20 $O/p2.log; exit 1; }
python3 scripts/r03/pmc_dispatch.py $O/p1 correspond_kernel | head -3
python3 scripts/r03/pmc_dispatch.py $O/p2 correspond_kernel | head -3
python3 scripts/r03/pmc_dispatch.py $O/p1 fdf_soa_kernel | head -1
find $O -name "*.csv" -size +20M -delete
echo done

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02/gtrace2; mkdir -p $O
B="python -u bench.py --steps 20 --warmup 2 --cpu-sample 0 --oracle-full 0 --fod-cpu-sample 0 --gn-steps 0 --no-events"
for cfg in "1 0" "1 1" "8 0" "8 1" "1 0" "1 1"; do set -- $cfg
 MGICP_GATE_POLLERS=$1 MGICP_MAIL_UNCACHED=$2 timeout -k 10 200 $B > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail $O/b_$1_$2.err; exit 1; }
 echo "pollers=$1 uncached=$2 $(python -c "import json;d=json.load(open('$O/b_$1_$2.json'));print(d['value'],d['ms_per_step'])")"
done
MGICP_GATED=0 timeout -k 10 200 $B > $O/b_plain.json 2> $O/b_plain.err && echo "plain $(python -c "import json;d=json.load(open('$O/b_plain.json'));print(d['value'],d['ms_per_step'])")"

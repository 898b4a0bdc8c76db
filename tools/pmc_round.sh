#!/bin/bash
# Counter round on the C2 bench (GPU box): kernel-trace stats, two SQ/GRBM passes
# (MFMA busy, issue/wait split, instruction mix, clock), FETCH_SIZE and WRITE_SIZE in
# separate passes.
# Every pass is its own rocprofv3 run under a time limit; counters the box does not
# list are dropped before a pass runs.  Usage: bash tools/pmc_round.sh TAG [bench args]
set -eo pipefail
TAG=${1:-cur}
shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --timer-steps 1 $*"
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
# the library build these counters belong to (bench.py reads PMC traffic only for its own build)
cp $R/cope-nerf_amd/copenerf/libcopenerf.so.stamp $O/lib_stamp.txt
have() { for c in "$@"; do grep -qw "$c" $O/counters.txt && printf '%s ' "$c"; done; }
echo "pass1: $(have SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT)"
echo "pass2: $(have SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks -o run --output-format csv -- $B > $O/bench_trace.json
P1=$(have SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT)
timeout -s KILL 300 rocprofv3 --pmc $P1 -d $O/p1 -o p1 --output-format csv -- $B > /dev/null
P2=$(have SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM)
timeout -s KILL 300 rocprofv3 --pmc $P2 -d $O/p2 -o p2 --output-format csv -- $B > /dev/null
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- $B > /dev/null
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- $B > /dev/null
python3 $R/tools/sq_summary.py $O/p1/p1_counter_collection.csv $O/p2/p2_counter_collection.csv > $O/sq_summary.txt
python3 $R/tools/pmc_summary.py $O/pf/run_counter_collection.csv $O/pw/run_counter_collection.csv $O/pmc.json
echo done

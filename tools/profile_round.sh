#!/bin/bash
# Kernel-trace stats + HBM traffic (FETCH_SIZE / WRITE_SIZE in separate --pmc
# passes) of the C2 bench; summaries land in gpurun_out/prof/ for copying into
# profiles/.  Usage (GPU box): bash tools/profile_round.sh TAG
set -e
TAG=${1:-cur}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_under_trace.json
cp $O/ks/run_kernel_stats.csv $O/${TAG}_kernel_stats.csv
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null
python3 $R/tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/${TAG}_pmc.json
timeout -k 10 300 python3 $R/bench.py > $O/${TAG}_bench.json

#!/bin/bash
# c3fp32 (Co3D stage 1, fp32-accurate) on the final tree: kernel-trace stats + its bench line.
set -eo pipefail
mkdir -p gpurun_out/s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s/ks -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c3fp32 --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/s/c3fp32_trace.json
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --config c3fp32 --no-cpu-baseline > gpurun_out/s/c3fp32_bench.json
tail -c 300 gpurun_out/s/c3fp32_bench.json

#!/bin/bash
# Round-3 final-kernel evidence: whole GPU suite + smoke, the counter round (kernel stats, SQ/GRBM,
# FETCH/WRITE), and the default bench line (with its CPU baseline).
set -eo pipefail
bash tools/gpu_suite.sh
WGRAD_VARIANTS=0 bash tools/pmc_round.sh r3o
timeout -k 10 300 python3 bench.py > gpurun_out/r3o_bench.json
tail -c 600 gpurun_out/r3o_bench.json

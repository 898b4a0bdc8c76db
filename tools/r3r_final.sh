#!/bin/bash
# Final tree check: the whole GPU suite + smoke, then the default bench line.
set -eo pipefail
bash tools/gpu_suite.sh
timeout -k 10 300 python3 bench.py > gpurun_out/r3r_bench.json
tail -c 400 gpurun_out/r3r_bench.json

#!/bin/bash
# Batched weight gradient: kernel test, then a same-box A/B of the C2 step (COPENERF_WGRAD_BATCH=0 / 1).
set -eo pipefail
mkdir -p gpurun_out/wb
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -s tests/test_gpu_x6.py -k batch > gpurun_out/wb/tests2.log 2>&1
tail -n 2 gpurun_out/wb/tests2.log
ARMS="nobatch=COPENERF_WGRAD_BATCH=0;batch=COPENERF_WGRAD_BATCH=1" REPS=3 bash tools/env_ab.sh

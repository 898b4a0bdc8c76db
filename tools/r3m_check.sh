#!/bin/bash
# Fused Adam (COPENERF_FUSED_ADAM): trainer / config / stage-1 / dist tests, then a same-box A/B of the C2 step.
set -eo pipefail
mkdir -p gpurun_out/m
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_configs.py tests/test_gpu_stage1.py tests/test_gpu_dist.py tests/test_gpu_evaluation.py > gpurun_out/m/tests.log 2>&1
tail -n 1 gpurun_out/m/tests.log
ARMS="foreach=COPENERF_FUSED_ADAM=0;fused=COPENERF_FUSED_ADAM=1" REPS=3 bash tools/env_ab.sh

#!/bin/bash
# ReLU sign-bit masks: the bitwise test, field/render/trainer tests with masks on, same-box A/B, kernel trace;
# then the whole default GPU suite + smoke on this tree.
set -eo pipefail
mkdir -p gpurun_out/u
timeout -k 10 150 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py -k sign_bit > gpurun_out/u/mask.log 2>&1
tail -n 1 gpurun_out/u/mask.log
COPENERF_RELU_MASK=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_render.py tests/test_gpu_trainer.py tests/test_gpu_raygrad.py > gpurun_out/u/tests.log 2>&1
tail -n 1 gpurun_out/u/tests.log
ARMS="act=COPENERF_RELU_MASK=0;mask=COPENERF_RELU_MASK=1" REPS=3 bash tools/env_ab.sh
bash tools/gpu_suite.sh

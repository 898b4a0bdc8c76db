#!/bin/bash
# Split-output MUL on the 256x256 tile: kernel + field/render/trainer tests, same-box A/B
# (COPENERF_SQ_NOSPLIT=1: the 128x256 tile), then every bench config on one box.
set -eo pipefail
mkdir -p gpurun_out/k
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_kernels.py tests/test_gpu_render.py tests/test_gpu_raygrad.py tests/test_gpu_stage1.py > gpurun_out/k/tests.log 2>&1
tail -n 1 gpurun_out/k/tests.log
ARMS="tall=COPENERF_SQ_NOSPLIT=1;sq=COPENERF_SQ_NOSPLIT=0" REPS=3 bash tools/env_ab.sh
bash tools/r3j_configs.sh

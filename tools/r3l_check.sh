#!/bin/bash
# SOFTPLUS_HEAD on the 256x256 tile's direct epilogue: kernel / field / render / trainer / stage-1 /
# config tests, then a same-box A/B against the 128x256 tile (COPENERF_X6_SQ=0x5f).
set -eo pipefail
mkdir -p gpurun_out/l
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_x6.py tests/test_gpu_render.py tests/test_gpu_trainer.py tests/test_gpu_stage1.py tests/test_gpu_configs.py tests/test_gpu_inference.py > gpurun_out/l/tests.log 2>&1
tail -n 1 gpurun_out/l/tests.log
ARMS="tall=COPENERF_X6_SQ=0x5f;sq=COPENERF_X6_SQ=0x15f" REPS=3 bash tools/env_ab.sh

#!/bin/bash
# Fused-encoding first layer on the 128x128 vs the 256x256 tile (batched weight gradients on in all
# arms but the first): same-box A/B of the C2 step, plus the bitwise test on the 256x256 variant.
set -eo pipefail
mkdir -p gpurun_out/g2
COPENERF_EMB_SQ=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py -k fused > gpurun_out/g2/tests.log 2>&1
tail -n 1 gpurun_out/g2/tests.log
ARMS="none=COPENERF_WGRAD_BATCH=0,COPENERF_FUSE_EMB=0;batch=COPENERF_WGRAD_BATCH=1,COPENERF_FUSE_EMB=0;embsq=COPENERF_WGRAD_BATCH=1,COPENERF_FUSE_EMB=1,COPENERF_EMB_SQ=1" REPS=3 bash tools/env_ab.sh

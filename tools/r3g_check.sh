#!/bin/bash
# Batched weight gradient + fused first-layer encoding: kernel tests, then a same-box A/B of the
# C2 step over the two knobs (COPENERF_WGRAD_BATCH, COPENERF_FUSE_EMB).
set -eo pipefail
mkdir -p gpurun_out/g
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -s tests/test_gpu_x6.py > gpurun_out/g/tests.log 2>&1
tail -n 2 gpurun_out/g/tests.log
ARMS="none=COPENERF_WGRAD_BATCH=0,COPENERF_FUSE_EMB=0;batch=COPENERF_WGRAD_BATCH=1,COPENERF_FUSE_EMB=0;emb=COPENERF_WGRAD_BATCH=0,COPENERF_FUSE_EMB=1;both=COPENERF_WGRAD_BATCH=1,COPENERF_FUSE_EMB=1" REPS=3 bash tools/env_ab.sh

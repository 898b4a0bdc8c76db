#!/bin/bash
# The whole GPU suite with every opt-in path of round 3 switched on at once (fused first-layer encoding,
# the SOFTPLUS layer chain, BWD_SOFTPLUS on the 128x256 two-per-CU tile).
set -eo pipefail
mkdir -p gpurun_out/t
COPENERF_FUSE_EMB=1 COPENERF_LAYER_CHAIN=1 COPENERF_X6_T2W=0x20 timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/tests.log 2>&1
tail -n 1 gpurun_out/t/tests.log

#!/bin/bash
# The 4x4 chain kernel (cn_mat4_chain) vs torch matmuls: GPU stage-1 tests, then c3fp32 A/B.
mkdir -p gpurun_out/cab
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage1_fused.py tests/test_gpu_stage1.py tests/test_gpu_configs.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/cab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/cab/tests.log
case $rc in 0) ;; *) exit $rc ;; esac
rm -f gpurun_out/env_ab/res.jsonl
ARMS="kernel=;torch=COPENERF_CHAIN_KERNEL=0" REPS=3 CONFIG=c3fp32 bash tools/env_ab.sh

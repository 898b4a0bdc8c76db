#!/bin/bash
# Row rounds on the 2-per-CU 128x128 tile (COPENERF_T128_ROUNDS=1): GPU parity tests with it on,
# then a same-box bench A/B, then its PMC HBM bytes for the BWD_SOFTPLUS class.
mkdir -p gpurun_out/rab
COPENERF_T128_ROUNDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_x6.py \
  tests/test_gpu_render.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/rab/tests.log
case $rc in 0) ;; *) exit $rc ;; esac
rm -f gpurun_out/env_ab/res.jsonl
ARMS="base=;rounds=COPENERF_T128_ROUNDS=1" REPS=3 bash tools/env_ab.sh

#!/bin/bash
# GPU tests touching the changed kernels, then a same-box A/B of the bench against a previous
# library build (ab/libcopenerf_prev.so, COPENERF_LIB) interleaved REPS times.
mkdir -p gpurun_out/lab
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_x6.py tests/test_gpu_render.py \
  tests/test_gpu_inference.py tests/test_gpu_trainer.py tests/test_gpu_stage1.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/lab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/lab/tests.log
case $rc in 0) ;; *) exit $rc ;; esac
rm -f gpurun_out/env_ab/res.jsonl
ARMS="new=;prev=COPENERF_LIB=$GRAFT_REPO_ROOT/ab/libcopenerf_prev.so" REPS=${REPS:-3} CONFIG=${CONFIG:-c2} bash tools/env_ab.sh

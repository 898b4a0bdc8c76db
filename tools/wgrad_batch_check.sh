#!/bin/bash
# GPU check of the batched weight gradient: kernel tests + trainer/render parity, then a same-box
# A/B of the C2 step with COPENERF_WGRAD_BATCH=0 / 1 and a kernel-trace of the batched step.
set -eo pipefail
mkdir -p gpurun_out/wb
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -s \
  tests/test_gpu_x6.py tests/test_gpu_kernels.py tests/test_gpu_render.py tests/test_gpu_trainer.py \
  tests/test_gpu_stage1.py tests/test_gpu_configs.py > gpurun_out/wb/tests.log 2>&1
tail -n 2 gpurun_out/wb/tests.log
ARMS="nobatch=COPENERF_WGRAD_BATCH=0;batch=COPENERF_WGRAD_BATCH=1" REPS=3 bash tools/env_ab.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/wb/ks -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/wb/bench_trace.json

#!/bin/bash
# Narrow (256x64) stage-ring weight gradient: kernel + field tests, same-box A/B of the C2 step
# (COPENERF_WGRAD_NARROW=0 / 1), kernel trace of the default step.
set -eo pipefail
mkdir -p gpurun_out/h
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_kernels.py tests/test_gpu_render.py > gpurun_out/h/tests.log 2>&1
tail -n 1 gpurun_out/h/tests.log
ARMS="old=COPENERF_WGRAD_NARROW=0;narrow=COPENERF_WGRAD_NARROW=1" REPS=3 bash tools/env_ab.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/h/ks -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/h/bench_trace.json

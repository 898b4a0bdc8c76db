#!/bin/bash
# Layer chain (cn_linear_chain): the bitwise test alone first (new kernel), then the field / render /
# trainer / config tests with the chain on, then a same-box A/B of the C2 step and a kernel trace.
set -eo pipefail
mkdir -p gpurun_out/q
timeout -k 10 150 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py -k chain > gpurun_out/q/chain.log 2>&1
tail -n 1 gpurun_out/q/chain.log
COPENERF_LAYER_CHAIN=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_render.py tests/test_gpu_trainer.py tests/test_gpu_configs.py tests/test_gpu_inference.py > gpurun_out/q/tests.log 2>&1
tail -n 1 gpurun_out/q/tests.log
ARMS="off=COPENERF_LAYER_CHAIN=0;chain=COPENERF_LAYER_CHAIN=1" REPS=3 bash tools/env_ab.sh
cd /tmp && export TMPDIR=/tmp
COPENERF_LAYER_CHAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/q/ks -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/q/bench_trace.json

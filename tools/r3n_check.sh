#!/bin/bash
# BWD_SOFTPLUS on the 128x256 two-per-CU tile (single-buffered B; COPENERF_X6_T2W=0x20): tests with it on,
# then a same-box A/B of the C2 step against the 128x128 tile, and a kernel trace of the T2W step.
set -eo pipefail
mkdir -p gpurun_out/n
COPENERF_X6_T2W=0x20 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_kernels.py tests/test_gpu_render.py tests/test_gpu_trainer.py > gpurun_out/n/tests.log 2>&1
tail -n 1 gpurun_out/n/tests.log
ARMS="t128=COPENERF_X6_T2W=0;t2w=COPENERF_X6_T2W=0x20" REPS=3 bash tools/env_ab.sh
cd /tmp && export TMPDIR=/tmp
COPENERF_X6_T2W=0x20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/n/ks -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/n/bench_trace.json

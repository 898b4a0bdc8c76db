#!/bin/bash
# Fused stage-1 pass: GPU parity tests, then a kernel-trace profile of the c3fp32 bench
# (only the per-kernel stats are kept: the full trace exceeds what gpurun copies back).
mkdir -p gpurun_out/s1b
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage1_fused.py tests/test_gpu_stage1.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s1b/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 124|134|137|139) exit $rc ;; esac
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/s1prof -o c3fp32 --output-format csv -- python bench.py --config c3fp32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/s1b/bench_trace.json 2> gpurun_out/s1b/bench_trace.err
rc=$?; echo "prof rc=$rc"
find /tmp/s1prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/s1b/ \;
find /tmp/s1prof -name '*kernel_trace.csv' -exec sh -c 'tail -n 20000 "$1" > gpurun_out/s1b/kernel_trace_tail.csv' _ {} \;
exit $rc

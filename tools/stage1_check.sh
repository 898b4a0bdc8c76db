#!/bin/bash
# Fused stage-1 pass check (GPU box): kernel + trainer parity tests, then the C3 stage-1
# bench lines with the fused pass and with the torch expressions (COPENERF_STAGE1_FUSED=0).
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stage1_fused.py tests/test_gpu_stage1.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/s1/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 124|134|137|139) exit $rc ;; esac
for c in ${CONFIGS:-c3fp32 c3}; do
  for f in 1 0; do
    COPENERF_STAGE1_FUSED=$f timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/s1/bench_${c}_f$f.json 2> gpurun_out/s1/bench_${c}_f$f.err || { echo "bench $c f$f failed"; exit 1; }
  done
done

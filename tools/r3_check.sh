#!/bin/bash
# Round-3 GPU check (GPU box): stage-1 / trainer / render parity tests (measured parity errors
# to gpurun_out/parity.jsonl), the autograd-liveness diagnostic, the C3 / C2 bench lines.
mkdir -p gpurun_out/r3c
COPENERF_PARITY_LOG=gpurun_out/r3c/parity.jsonl timeout -k 10 800 python -u -m pytest tests/test_gpu_stage1.py \
  tests/test_gpu_trainer.py tests/test_gpu_render.py tests/test_gpu_configs.py -q --timeout 300 --timeout-method thread > gpurun_out/r3c/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 120 python tools/graph_alive.py --stage1 > gpurun_out/r3c/alive.log 2>&1 || echo "alive rc=$?"
for c in ${CONFIGS:-c3fp32 c3 c3pose c2}; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3c/bench_$c.json 2> gpurun_out/r3c/bench_$c.err || { echo "bench $c failed"; break; }
done

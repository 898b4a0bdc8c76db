#!/bin/bash
# Weight gradients on a side stream (COPENERF_WGRAD_STREAM=1) vs serial: GPU parity tests with
# the side stream on, then same-box bench A/B (eager C2, graph-captured C2, C3 stage 1).
mkdir -p gpurun_out/sab
for arm in 0 1 0 1; do
  for c in c2 c2g c3fp32; do
    a="--config $c"; [ $c = c2g ] && a="--config c2 --graph"
    COPENERF_WGRAD_STREAM=$arm timeout -k 10 200 python bench.py $a --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/sab/${c}_$arm.json 2> gpurun_out/sab/${c}_$arm.err || { echo "bench $c $arm failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/sab/${c}_$arm.json').read().strip().splitlines()[-1]); print('$c arm $arm', d['value'], d['ms_per_step'])"
  done
done

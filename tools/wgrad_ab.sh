#!/bin/bash
# A/B of the 256x256 bf16x6 weight-gradient kernels (tools/wgrad_ab.py), each variant in its
# own process, interleaved twice; LIBS: extra library builds to compare (COPENERF_LIB paths)
set -eo pipefail
mkdir -p gpurun_out/wab
for rep in $(seq ${REPS:-2}); do
  for lib in cope-nerf_amd/copenerf/libcopenerf.so $LIBS; do
    for v in ${VARIANTS:-0 1 2 3 4}; do
      COPENERF_LIB=$lib COPENERF_WGRAD_KERNEL=$v timeout -k 10 120 python tools/wgrad_ab.py | tee -a gpurun_out/wab/res.jsonl
    done
  done
done

#!/bin/bash
# C2 step time against rays per step (is per-ray cost lower at smaller M? the memory-side
# cache holds a 262k-row activation, not a 524k-row one)
mkdir -p gpurun_out/rs
for r in 1024 2048 4096 8192; do
  timeout -k 10 200 python bench.py --config c2 --rays $r --steps 10 --warmup 3 --no-cpu-baseline --timer-steps 0 \
    > gpurun_out/rs/r$r.json 2> gpurun_out/rs/r$r.err || { echo "rays $r failed"; exit 1; }
done

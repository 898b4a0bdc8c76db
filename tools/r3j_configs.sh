#!/bin/bash
# Every bench config on one box on the final round-3 kernels, then the verdict's BWD_SOFTPLUS-on-
# the-256x256-tile default candidate (COPENERF_X6_SQ=0x7f) A/B'd against the current 0x5f.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3j
mkdir -p $O
for c in c2graph c2fp32 c2bf16 c3 c3fp32 c3pose c4 c5 infer distgraph; do
  case $c in
    c2graph) args="--graph";;
    distgraph) args="--graph"; export COPENERF_FORCE_DIST=1;;
    *) args="--config $c";;
  esac
  timeout -k 10 400 python3 -u $R/bench.py $args --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed rc=$?"; tail -5 $O/bench_$c.err; exit 1; }
  unset COPENERF_FORCE_DIST
  python3 -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'])"
done
ARMS="sq5f=COPENERF_X6_SQ=0x5f;sq7f=COPENERF_X6_SQ=0x7f" REPS=3 bash tools/env_ab.sh

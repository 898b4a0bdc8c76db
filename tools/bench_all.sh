#!/bin/bash
# Every bench.py config on one GPU (+ the 1-rank RCCL graph path) and the rocprofv3
# kernel-trace summary of the headline; results in gpurun_out/<tag>/.  GPU box only.
#   bash tools/bench_all.sh TAG [configs...]
set -o pipefail
TAG=${1:-cur}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
CONFIGS=${@:-"c2 c2graph c3 c3fp32 c4 c5 distgraph"}
for c in $CONFIGS; do
  case $c in
    c2) args="";;
    c2graph) args="--graph --no-cpu-baseline";;
    distgraph) args="--graph --no-cpu-baseline"; export COPENERF_FORCE_DIST=1;;
    *graph) args="--config ${c%graph} --graph --no-cpu-baseline";;
    *) args="--config $c";;
  esac
  echo "== $c $args" >&2
  timeout -k 10 400 python3 -u $R/bench.py $args > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed rc=$?" >&2; tail -5 $O/bench_$c.err >&2; exit 1; }
  unset COPENERF_FORCE_DIST
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['bound'], r['achieved'], r['unit'], r['frac'])" >&2
done

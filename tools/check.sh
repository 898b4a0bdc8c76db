#!/bin/bash
# One GPU-box check of the tree: the GPU test suite in one process (optional), smoke(), then
# bench.py lines for the given configs.  Results in gpurun_out/<tag>/.  Every GPU step runs under
# its own time limit and the first failure ends the script (no retries).
#   bash tools/check.sh TAG [--no-tests] [configs...]     (configs default: c2)
set -o pipefail
TAG=${1:-cur}; shift
TESTS=1
if [ "$1" = "--no-tests" ]; then TESTS=0; shift; fi
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ $TESTS = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.txt
  [ $rc = 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.txt
  [ $rc = 0 ] || exit $rc
fi
for c in ${@:-c2}; do
  # <config>graph: the config replayed from a captured HIP graph
  # distgraph: c2 through the data-parallel path (a 1-rank RCCL group, graph-captured all-reduce)
  case $c in distgraph) args="--config c2 --graph"; export COPENERF_FORCE_DIST=1;;
             *graph) args="--config ${c%graph} --graph";; *) args="--config $c";; esac
  timeout -k 10 400 python3 -u bench.py $args --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  rc=$?
  unset COPENERF_FORCE_DIST
  [ $rc = 0 ] || { echo "bench $c failed rc=$rc"; tail -5 $O/bench_$c.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['launch_class'], d['roofline']['frac'])"
done
echo done

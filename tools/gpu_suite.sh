#!/bin/bash
# The whole GPU suite in one process (the driver's round-end tier), then smoke().
mkdir -p gpurun_out/suite
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/suite/tests.log
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1
echo "smoke rc=$?"

#!/bin/bash
# Test-pose optimisation (eval.py:44-93) GPU tests.
mkdir -p gpurun_out/ev
timeout -k 10 400 python -u -m pytest tests/test_gpu_evaluation.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/ev/tests.log 2>&1
echo "tests rc=$?"

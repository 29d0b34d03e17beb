#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sep
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sep/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sep/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/sep/pytest_gpu.txt
HRF_REG_SEPARABLE=0 timeout -k 10 200 python -u -m pytest tests/test_registration_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sep/pytest_reg0.txt 2>&1 || { echo "reg tests (2-D plans) failed"; tail -30 gpurun_out/sep/pytest_reg0.txt; exit 1; }
tail -1 gpurun_out/sep/pytest_reg0.txt
AB_REPS=3 timeout -k 10 700 bash tools/bench_ab.sh HRF_REG_SEPARABLE=0 HRF_REG_SEPARABLE=1 && cat gpurun_out/ab.log

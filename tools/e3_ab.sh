#!/bin/bash
# enhance3d: parity tests, then timing per variant (env)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_enhance_gpu.py > gpurun_out/e3_test.txt 2>&1
HRF_E3_WPE=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_enhance_gpu.py >> gpurun_out/e3_test.txt 2>&1
: > gpurun_out/e3_time.txt
for v in "$@"; do
  echo "== $v" >> gpurun_out/e3_time.txt
  env $v timeout -k 10 120 python tools/time_kernels.py enhance3d >> gpurun_out/e3_time.txt 2>&1
done

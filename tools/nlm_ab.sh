#!/bin/bash
# NL-means kernel A/B on one box: parity tests, then each variant's 2048^2 timing
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nlmeans_gpu.py > gpurun_out/nlm_test.txt 2>&1
: > gpurun_out/nlm_time.txt
for v in "$@"; do
  echo "== $v" >> gpurun_out/nlm_time.txt
  env $v timeout -k 10 120 python tools/time_kernels.py nlmeans >> gpurun_out/nlm_time.txt 2>&1
done

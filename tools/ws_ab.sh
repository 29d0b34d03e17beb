#!/bin/bash
# watershed tie path: tests, then the adversarial timing per scratch budget
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_watershed_gpu.py > gpurun_out/ws_test.txt 2>&1
tail -1 gpurun_out/ws_test.txt
: > gpurun_out/ws_time.txt
for v in "$@"; do
  echo "== $v" >> gpurun_out/ws_time.txt
  env $v timeout -k 10 150 python tools/time_ws_ties.py >> gpurun_out/ws_time.txt 2>&1
done
grep -v amdgpu.ids gpurun_out/ws_time.txt

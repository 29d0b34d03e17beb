#!/bin/bash
# lasers label sums: reciprocal vs per-channel division, alternating, on one box
set -e
: > gpurun_out/lsl_ab.txt
for i in 1 2 3; do
  for v in "HRF_LSL_X=0" "HRF_LSL_DIV=1"; do
    echo "== $v" >> gpurun_out/lsl_ab.txt
    env $v timeout -k 10 120 python tools/time_kernels.py path 2>&1 | grep label_sums >> gpurun_out/lsl_ab.txt
  done
done

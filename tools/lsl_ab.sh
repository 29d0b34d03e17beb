#!/bin/bash
# lasers label sums, isolated (time_kernels.py path), alternating environment settings on one box
# usage: bash tools/lsl_ab.sh "<env 1>" "<env 2>" ...   (default: the row-chunk kernel vs the general one)
set -e
: > gpurun_out/lsl_ab.txt
[ $# -eq 0 ] && set -- "HRF_LSL_X=0" "HRF_LSL_ROW=0"
for i in 1 2 3; do
  for v in "$@"; do
    echo "== $v" >> gpurun_out/lsl_ab.txt
    env $v timeout -k 10 120 python tools/time_kernels.py path 2>&1 | grep label_sums >> gpurun_out/lsl_ab.txt
  done
done

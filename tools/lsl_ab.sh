#!/bin/bash
# lasers label sums, isolated (time_kernels.py path), alternating environment settings on one box
# usage: bash tools/lsl_ab.sh "<env 1>" "<env 2>" ...   (e.g. HRF_LIB=ab/libhrf_<tag>.so against HRF_NONE=1)
set -e
: > gpurun_out/lsl_ab.txt
[ $# -eq 0 ] && { echo "usage: bash tools/lsl_ab.sh \"<env 1>\" \"<env 2>\" ..."; exit 2; }
for i in 1 2 3; do
  for v in "$@"; do
    echo "== $v" >> gpurun_out/lsl_ab.txt
    env $v timeout -k 10 120 python tools/time_kernels.py path 2>&1 | grep label_sums >> gpurun_out/lsl_ab.txt
  done
done

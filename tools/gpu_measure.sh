#!/bin/bash
# one box: enhance3d variants, NL-means, interleaved bench lines (env A/B)
set -o pipefail
mkdir -p gpurun_out/batch
o=gpurun_out/batch
: > $o/time.txt
for v in HRF_E3_WPE=2 HRF_E3_WPE=1; do
  echo "== $v" >> $o/time.txt
  env $v timeout -k 10 120 python tools/time_kernels.py enhance3d >> $o/time.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $o/time.txt
bash tools/bench_ab_envs.sh 3 - HRF_STREAM_GRID_MAX=512 || exit 1
tail -4 gpurun_out/ab_envs.log

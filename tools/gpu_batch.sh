#!/bin/bash
# one box: GPU suite (all, no -x), enhance3d variants, NL-means, two bench lines
set -o pipefail
mkdir -p gpurun_out/batch
o=gpurun_out/batch
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1
rc=$?
tail -3 $o/pytest.txt
case $rc in 0|1) ;; *) echo "test run ended with status $rc"; exit 1;; esac
for v in HRF_E3_WPE=1 HRF_E3_WPE=2; do
  echo "== $v" >> $o/time.txt
  env $v timeout -k 10 120 python tools/time_kernels.py enhance3d >> $o/time.txt 2>&1 || exit 1
done
timeout -k 10 120 python tools/time_kernels.py nlmeans >> $o/time.txt 2>&1 || exit 1
grep -v amdgpu.ids $o/time.txt
bash tools/bench_ab_envs.sh 2 - HRF_STREAM_GRID_MAX=512 || exit 1
cat gpurun_out/ab_envs.log | tail -3

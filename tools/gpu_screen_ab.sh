#!/bin/bash
# screen-kernel variants: the exact-path timing of each ab/ build, then interleaved bench runs
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-scr}
mkdir -p $o
for v in ab/libhrf_*.so; do
  HRF_LIB=$PWD/$v timeout -k 10 200 python -u tools/time_classify_exact.py > $o/time_$(basename $v .so).txt 2>&1 || { echo "timing $v failed"; exit 1; }
  echo "$v: $(grep screen $o/time_$(basename $v .so).txt | head -1)"
done
timeout -k 10 200 python -u tools/time_classify_exact.py > $o/time_default.txt 2>&1 || { echo "timing failed"; exit 1; }
echo "default: $(grep screen $o/time_default.txt | head -1)"
envs=("-")
for v in ab/libhrf_*.so; do envs+=("HRF_LIB=$PWD/$v"); done
bash tools/bench_ab_envs.sh ${2:-2} "${envs[@]}"

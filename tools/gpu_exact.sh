#!/bin/bash
# exact per-pixel classifier: its tests, then the screen / refine timing (default build and the
# A/B variants in ab/).  usage: bash tools/gpu_exact.sh <tag> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r6}
o=gpurun_out/$tag
mkdir -p $o
k=${2:-}
timeout -k 10 600 python -u -m pytest tests/test_classify_exact_gpu.py tests/test_kernels_gpu.py tests/test_regtile_gpu.py \
  -m gpu -x -v --timeout 300 --timeout-method thread ${k:+-k "$k"} > $o/pytest.txt 2>&1
rc=$?
tail -5 $o/pytest.txt
case $rc in 0|1) ;; *) echo "test run ended with status $rc"; exit 1;; esac
timeout -k 10 200 python -u tools/time_classify_exact.py > $o/time_default.txt 2>&1 || { echo "timing failed"; tail $o/time_default.txt; exit 1; }
cat $o/time_default.txt
for v in ab/libhrf_*.so; do
  [ -e "$v" ] || continue
  HRF_LIB=$v timeout -k 10 200 python -u tools/time_classify_exact.py > $o/time_$(basename $v .so).txt 2>&1 || { echo "timing $v failed"; exit 1; }
  echo "$v: $(head -1 $o/time_$(basename $v .so).txt)"
done

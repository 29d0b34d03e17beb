#!/bin/bash
# exact classifier: quick tests, timing, and the kernel-trace stats of the timing run
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r6}
lib=${2:-}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_classify_exact_gpu.py tests/test_kernels_gpu.py -k "classif" -m gpu -x -q \
  --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1
rc=$?
tail -3 $o/pytest.txt
case $rc in 0) ;; *) echo "tests ended with status $rc"; exit 1;; esac
export HRF_LIB=$lib
timeout -k 10 200 python -u tools/time_classify_exact.py > $o/time.txt 2>&1 || { echo "timing failed"; tail $o/time.txt; exit 1; }
grep -v amdgpu.ids $o/time.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 tools/time_classify_exact.py 5 > $o/prof.txt 2>&1 || { echo "prof failed"; tail $o/prof.txt; exit 1; }
f=$(find $o/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | head -12

#!/bin/bash
# exact classifier: quick tests on the default build, then the timing of every ab/ variant
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r6}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_classify_exact_gpu.py tests/test_kernels_gpu.py tests/test_regtile_gpu.py tests/test_tile_gpu.py -k "classif or regtile or tile or assembly" -m gpu -x -q \
  --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1
rc=$?
tail -3 $o/pytest.txt
case $rc in 0) ;; *) echo "tests ended with status $rc"; exit 1;; esac
for rep in 1 2; do
  timeout -k 10 200 python -u tools/time_classify_exact.py > $o/time_default_$rep.txt 2>&1 || { echo "timing failed"; exit 1; }
  echo "default: $(grep screen $o/time_default_$rep.txt | head -1)"
  for v in ab/libhrf_*.so; do
    [ -e "$v" ] || continue
    HRF_LIB=$PWD/$v timeout -k 10 200 python -u tools/time_classify_exact.py > $o/time_$(basename $v .so)_$rep.txt 2>&1 || { echo "timing $v failed"; exit 1; }
    echo "$v: $(grep screen $o/time_$(basename $v .so)_$rep.txt | head -1)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 tools/time_classify_exact.py 5 > $o/prof.txt 2>&1 || { echo "prof failed"; exit 1; }
python3 - "$o" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/*kernel_stats.csv")[0]
for r in list(csv.DictReader(open(f)))[:4]:
    print("%-60s %4s calls %.3f ms avg" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY

#!/bin/bash
# kernel trace of the default concurrent bench + the concurrency picture.  usage: bash tools/gpu_concprof.sh <tag> [bench args]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-conc}; shift
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/tr -o run -- python3 bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline "$@" > $o/bench.json 2> $o/err.txt || { echo "profile failed"; tail -5 $o/err.txt; exit 1; }
cut -c1-160 $o/bench.json
f=$(find $o/tr -name '*kernel_trace.csv' | head -1)
python3 tools/conc_analysis.py "$f" ${CONC_MARK:-classify_pixels} > $o/conc.txt && cat $o/conc.txt
python3 tools/trace_summary.py "$f" ${CONC_MARK:-classify_pixels} 40 > $o/summary.txt && cat $o/summary.txt

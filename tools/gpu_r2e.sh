#!/bin/bash
# isolated segmentation kernel profile + priority A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2e
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e/seg -o seg -- python3 tools/prof_segment.py > gpurun_out/r2e/prof_segment.txt 2>&1 || { echo "prof_segment failed"; tail -20 gpurun_out/r2e/prof_segment.txt; exit 1; }
cat gpurun_out/r2e/prof_segment.txt
AB_REPS=3 timeout -k 10 900 bash tools/bench_ab.sh HRF_PRIORITY=1 HRF_PRIORITY=2 || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log gpurun_out/r2e/ab_priority.log
cat gpurun_out/r2e/ab_priority.log

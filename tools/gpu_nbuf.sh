#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/nbuf
HRF_CLASSIFY_NBUF=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q -k "classify or process_tile or concurrent or seeds" --timeout 200 --timeout-method thread > gpurun_out/nbuf/pytest2.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/nbuf/pytest2.txt; exit 1; }
tail -1 gpurun_out/nbuf/pytest2.txt
AB_REPS=3 timeout -k 10 700 bash tools/bench_ab.sh HRF_CLASSIFY_NBUF=3 HRF_CLASSIFY_NBUF=2 && cat gpurun_out/ab.log

#!/bin/bash
# classifier forms: parity subset under both MFMA shapes, isolated timings, PMC of the default
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/m16
mkdir -p $o
for m in 1 0; do
HRF_CLASSIFY_MFMA16=$m timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py tests/test_abi.py -m gpu -x -q -k "classify or process_tile or concurrent or abi" --timeout 200 --timeout-method thread > $o/pytest$m.txt 2>&1 || { echo "tests $m failed"; tail -40 $o/pytest$m.txt; exit 1; }
tail -1 $o/pytest$m.txt
HRF_CLASSIFY_MFMA16=$m timeout -k 10 120 python -u tools/time_kernels.py classify > $o/t$m.txt 2>&1 && grep "mode 2" $o/t$m.txt
done
bash tools/gpu_pmc.sh ${1:-m16} 2 || { echo "pmc failed"; exit 1; }

#!/bin/bash
# native-tile tests + A/B of the native tile call against the composed path
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tile_gpu.py tests/test_kernels_gpu.py -k "tile or kmeans or segment_flags or classify_cells" > gpurun_out/t_tile.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_tile.txt; exit 1; }
tail -2 gpurun_out/t_tile.txt
bash tools/bench_ab_envs.sh ${1:-2} "HRF_TILE_NATIVE=0" "HRF_TILE_NATIVE=1"

#!/bin/bash
# GPU round trip used during development: tests, bench, kernel-trace profile (csv).
set -o pipefail
export TMPDIR=/tmp
tag=${1:-dev}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t_$tag.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o trace -- python3 bench.py --steps 7 --warmup 2 > gpurun_out/prof_${tag}_bench.log 2>&1 || { echo "profile failed"; exit 1; }
echo done

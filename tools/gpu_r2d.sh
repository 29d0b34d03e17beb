#!/bin/bash
# Round-2 re-entry check: GPU suite, full bench line, kernel-trace stats of the same bench command.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r2d}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$tag/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/$tag/pytest_gpu.txt
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { echo "bench failed"; tail -30 gpurun_out/$tag/bench.err; exit 1; }
cat gpurun_out/$tag/bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run -- python3 bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/$tag/prof_bench.json 2> gpurun_out/$tag/prof.err || { echo "profile failed"; exit 1; }

mkdir -p gpurun_out/r2e
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e/seg -o seg -- python3 tools/prof_segment.py > gpurun_out/r2e/prof_segment.txt 2>&1 || { echo "prof_segment failed"; tail -20 gpurun_out/r2e/prof_segment.txt; exit 1; }
cat gpurun_out/r2e/prof_segment.txt
AB_REPS=2 timeout -k 10 500 bash tools/bench_ab.sh HRF_PRIORITY=1 HRF_PRIORITY=2 || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log gpurun_out/r2e/ab_priority.log
cat gpurun_out/r2e/ab_priority.log

#!/bin/bash
# Round profile: the full bench line, then the kernel-trace summary of the same command
# (shorter run) -- usage: bash tools/gpu_round_profile.sh <tag>
set -o pipefail
tag=${1:-r2}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run -- python3 bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/$tag/prof_bench.json 2> gpurun_out/$tag/prof.err

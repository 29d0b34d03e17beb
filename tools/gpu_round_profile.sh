#!/bin/bash
# Round-end evidence: full bench line, then a kernel-trace profile of the main workload.
# usage: bash tools/gpu_round_profile.sh <tag>   -> gpurun_out/<tag>_bench.json, gpurun_out/<tag>_kt/
set -o pipefail
export TMPDIR=/tmp
tag=${1:-rx}
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_kt -o kt -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/${tag}_kt.out 2> gpurun_out/${tag}_kt.err &&
echo done

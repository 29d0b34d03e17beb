#!/bin/bash
# kernel-trace of a short bench run (csv) -> gpurun_out/<tag>/prof
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-prof}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > $o/prof_bench.json 2> $o/prof.err || { echo "profile failed"; tail -5 $o/prof.err; exit 1; }
cut -c1-200 $o/prof_bench.json

#!/bin/bash
# interleaved A/B of two bench scripts -> gpurun_out/ab_bench.log
# usage: bash tools/ab_bench.sh <A.py> <B.py> [reps] [extra bench args]
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_bench.log
: > $out
A=$1; B=$2; reps=${3:-3}; shift 3
for r in $(seq $reps); do
  for s in $A $B; do
    v=$(timeout -k 10 240 python3 $s --no-cpu-baseline --no-extras "$@" 2>>gpurun_out/ab_bench.err) || exit 1
    echo "[$s $*] $(echo "$v" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')" >> $out
  done
done

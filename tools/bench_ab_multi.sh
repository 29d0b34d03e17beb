#!/bin/bash
# Interleaved A/B of environment settings under several bench argument sets.
# usage: bash tools/bench_ab_multi.sh <reps> "<env A>" "<env B>" "<args 1>" ["<args 2>" ...]
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_multi.log
: > $out
reps=$1; A=$2; B=$3; shift 3
for args in "$@"; do
  for rep in $(seq $reps); do
    for e in "$A" "$B"; do
      r=$(env $e timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 5 $args 2>/dev/null) || exit 1
      echo "[$e | $args] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("roofline", {}).get("kernel_ms"))')" >> $out
    done
  done
done
cat $out

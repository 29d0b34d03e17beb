#!/bin/bash
# A/B of two bench argument sets, interleaved: bash tools/bench_ab_args.sh "<args A>" "<args B>" [reps]
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_args.log
: > $out
A=$1; B=$2; reps=${3:-3}
for rep in $(seq $reps); do
  for a in "$A" "$B"; do
    r=$(timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 5 $a 2>/dev/null) || exit 1
    echo "[$a] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("roofline", {}).get("kernel_ms"))')" >> $out
  done
done

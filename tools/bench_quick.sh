#!/bin/bash
# default bench line + segmentation-only line -> gpurun_out/quick.log
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/quick.log
: > $out
for args in "" "--no-per-pixel"; do
  r=$(timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 $args 2>/dev/null) || exit 1
  echo "[$args] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
done

#!/bin/bash
# bench.py under a few concurrency / per-pixel settings (one line each) -> gpurun_out/variants.log
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/variants.log
: > $out
for args in "" "--no-per-pixel" "--concurrent 1" "--concurrent 3" "--concurrent 4" "--no-per-pixel --concurrent 4"; do
  r=$(timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 $args 2>/dev/null) || exit 1
  echo "[$args] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
done

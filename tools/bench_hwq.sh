#!/bin/bash
# bench.py at 2..4 concurrent tiles under GPU_MAX_HW_QUEUES 4 / 8 / 16 -> gpurun_out/hwq.log
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/hwq.log
: > $out
for rep in 1 2; do
for q in 4 8 16; do
for c in 2 3 4; do
  r=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 12 --warmup 4 --concurrent $c "$@" 2>/dev/null) || exit 1
  echo "[hwq $q concurrent $c $*] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')" >> $out
done; done; done

#!/bin/bash
# bench.py at 1..4 concurrent tiles -> gpurun_out/conc.log
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/conc.log
: > $out
for c in 2 3 4 2 3 4; do
  r=$(timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 12 --warmup 4 --concurrent $c "$@" 2>/dev/null) || exit 1
  echo "[concurrent $c $*] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
done

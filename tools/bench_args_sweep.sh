#!/bin/bash
# One bench line per argument set (value, ms/step, in-bench classifier ms).  usage: bash tools/bench_args_sweep.sh "<args 1>" "<args 2>" ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/args_sweep.log
: > $out
for a in "$@"; do
  r=$(timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 5 $a 2>/dev/null) || exit 1
  echo "[$a] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("roofline", {}).get("kernel_ms"))')" | tee -a $out
done

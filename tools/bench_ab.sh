#!/bin/bash
# A/B of an environment setting on the bench, interleaved: bash tools/bench_ab.sh "VAR=a" "VAR=b" [bench args]
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab.log
: > $out
A=$1; B=$2; shift 2
for rep in $(seq ${AB_REPS:-5}); do
  for e in "$A" "$B"; do
    r=$(env $e timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 "$@" 2>/dev/null) || exit 1
    echo "[$e $*] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("roofline", {}).get("kernel_ms"))')" >> $out
  done
done

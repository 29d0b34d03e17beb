#!/bin/bash
# Interleaved comparison of bench argument sets: bash tools/bench_ab_args.sh <reps> "<args A>" "<args B>" ...
# (leading NAME=value words of a set are put in the environment of that run)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_args.log
: > $out
reps=$1; shift
for rep in $(seq $reps); do
  for a in "$@"; do
    envs=(); args=()
    for w in $a; do
      if [ ${#args[@]} -eq 0 ] && [[ $w =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$w"); else args+=("$w"); fi
    done
    r=$(env HRF_NONE=1 "${envs[@]}" timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 5 "${args[@]}" 2>/dev/null) || exit 1
    echo "[$a] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("roofline", {}).get("kernel_ms"))')" >> $out
  done
done
python3 - "$out" <<'PY'
import collections, sys, re
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"\[(.*)\] (\S+)", line)
    if m: d[m.group(1)].append(float(m.group(2)))
for k, v in d.items(): print("%-40s mean %.1f  %s" % (k, sum(v) / len(v), v))
PY

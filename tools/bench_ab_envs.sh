#!/bin/bash
# Interleaved comparison of several environment settings on the default bench.
# usage: bash tools/bench_ab_envs.sh <reps> "<env 1>" "<env 2>" ...   (env "-" = none)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_envs.log
: > $out
reps=$1; shift
for rep in $(seq $reps); do
  for e in "$@"; do
    ev=$e; [ "$e" = "-" ] && ev="HRF_NONE=1"
    r=$(env $ev timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 5 2>/dev/null) || exit 1
    echo "[$e] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("roofline", {}).get("kernel_ms"))')" >> $out
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

#!/bin/bash
# tools/time_preassembled.py under alternating environment settings (e.g. HRF_LIB=ab/libhrf_<tag>.so)
# usage: bash tools/pre_ab.sh <reps> "<env 1>" "<env 2>" ...   (env "-" = none)
set -o pipefail
out=gpurun_out/pre_ab.log
: > $out
reps=$1; shift
for rep in $(seq $reps); do
  for e in "$@"; do
    ev=$e; [ "$e" = "-" ] && ev="HRF_NONE=1"
    r=$(env $ev timeout -k 10 240 python3 tools/time_preassembled.py 30 2>/dev/null | tail -1) || exit 1
    echo "[$e] $r" >> $out
  done
done
cat $out

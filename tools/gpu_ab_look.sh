#!/bin/bash
# lookahead A/B + the serial per-tile kernel trace of the bench path
set -o pipefail
export TMPDIR=/tmp
HRF_LOOKAHEAD=0 bash tools/gpu_seqprof.sh r3seq > /dev/null || exit 1
tail -45 gpurun_out/r3seq/seq_summary.txt
bash tools/bench_ab_envs.sh 3 "HRF_LOOKAHEAD=0" "HRF_LOOKAHEAD=1"

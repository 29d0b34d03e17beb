#!/bin/bash
# Sequential single-tile kernel traces (no concurrency, no overlap): each kernel's own duration
# per tile -- the CU-time budget of the path.  usage: bash tools/gpu_seqprof.sh <tag>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-seq}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/seq -o run -- python3 bench.py --concurrent 1 --no-overlap --steps 20 --warmup 3 --no-extras --no-cpu-baseline > $o/seq_bench.json 2> $o/seq.err || { echo "seq profile failed"; tail -5 $o/seq.err; exit 1; }
cut -c1-200 $o/seq_bench.json
f=$(find $o/seq -name '*kernel_trace.csv' | head -1)
python3 tools/trace_summary.py "$f" assemble_ecoli_kernel 45 > $o/seq_summary.txt && cat $o/seq_summary.txt

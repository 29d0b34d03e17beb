#!/bin/bash
# development round trip: GPU suite, stream-kernel timings, isolated segmentation, quick bench
set -o pipefail
export TMPDIR=/tmp
tag=${1:-it}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -40 $o/pytest_gpu.txt; exit 1; }
tail -1 $o/pytest_gpu.txt
timeout -k 10 200 python -u tools/time_kernels.py stream > $o/stream.txt 2>&1 || { echo "time_kernels failed"; tail -20 $o/stream.txt; exit 1; }
cat $o/stream.txt
timeout -k 10 200 python -u tools/prof_segment.py > $o/seg.txt 2>&1 || { echo "prof_segment failed"; tail -20 $o/seg.txt; exit 1; }
cat $o/seg.txt
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --steps 60 --warmup 5 > $o/bench$i.json 2> $o/bench$i.err || { echo "bench failed"; tail -20 $o/bench$i.err; exit 1; }
cut -c1-200 $o/bench$i.json
done
if [ -n "$PMC" ]; then bash tools/gpu_pmc_hbm.sh || { echo "pmc failed"; exit 1; }; fi

#!/bin/bash
# Wave-slot cost of every kernel of the timed path: SQ_WAVE_CYCLES (waves x cycles resident, the
# occupancy a kernel takes from the concurrent tiles) per kernel per tile, one tile at a time.
# usage: bash tools/gpu_wavecycles.sh <tag>; summarise with tools/wavecycles_table.py
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-wc}
mkdir -p $o
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $o/pmc -o pmc -- \
  python3 bench.py --concurrent 1 --no-overlap --steps 10 --warmup 2 --no-extras --no-cpu-baseline > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
f=$(find $o/pmc -name '*counter_collection.csv' | head -1)
python3 tools/wavecycles_table.py "$f" > $o/table.txt && head -50 $o/table.txt

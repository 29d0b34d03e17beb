#!/bin/bash
# PMC passes over the isolated classifier (tools/time_classify.py, R = 1023), one counter
# group per rocprofv3 run (gfx950 slot limits: 8 SQ, 4 TCC -- FETCH_SIZE 3, WRITE_SIZE 2).
# usage: bash tools/gpu_pmc.sh <tag> [mode]   (mode "t": the pixel-table kernel the bench times)
set -o pipefail
export TMPDIR=/tmp
tag=${1:-dev}
mode=${2:-2}
out=gpurun_out/pmc_$tag
mkdir -p $out
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o pmc -- \
    python3 tools/time_classify.py $mode 1023 > $out/$name.log 2>&1
}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- \
  python3 tools/time_classify.py $mode 1023 > $out/kt.log 2>&1 &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE &&
echo pmc done

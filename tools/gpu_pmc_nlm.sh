#!/bin/bash
# PMC passes over the NL-means kernel (tools/time_kernels.py nlmeans), one counter group per
# rocprofv3 run (HRF_LIB selects an A/B build).  usage: bash tools/gpu_pmc_nlm.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_nlm_$1
mkdir -p $out
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o pmc -- \
    python3 tools/time_kernels.py nlmeans > $out/$name.log 2>&1
}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- \
  python3 tools/time_kernels.py nlmeans > $out/kt.log 2>&1 &&
run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE &&
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM &&
echo pmc done

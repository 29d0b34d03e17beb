#!/bin/bash
# SQ counters of the timed path's streaming kernels (tools/time_kernels.py path): issue, wait and
# LDS behaviour of the assembly, the channel max and the label sums.  One counter group per run.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_path_sq
mkdir -p $out
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $out/sq1 -o pmc -- \
  python3 tools/time_kernels.py path > $out/sq1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --output-format csv -d $out/sq2 -o pmc -- \
  python3 tools/time_kernels.py path > $out/sq2.log 2>&1 &&
echo pmc done

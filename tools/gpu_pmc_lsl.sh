#!/bin/bash
# SQ counters of the lasers label sums variants (tools/time_kernels.py path) under the env
# settings given as arguments, one counter group per run; summarise with tools/pmc_table.py
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_lsl
mkdir -p $out
for v in "$@"; do
  tag=$(echo "$v" | tr -c 'A-Za-z0-9\n' '_')
  env $v timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $out/$tag.sq1 -o pmc -- \
    python3 tools/time_kernels.py path > $out/$tag.sq1.log 2>&1 || exit 1
  env $v timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --output-format csv -d $out/$tag.sq2 -o pmc -- \
    python3 tools/time_kernels.py path > $out/$tag.sq2.log 2>&1 || exit 1
done
echo pmc done

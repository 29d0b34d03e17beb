#!/bin/bash
# SQ counter passes over the isolated classifier for several HRF_CLASSIFY_W16 settings, plus a
# library-size scan (prologue vs sweep).  usage: bash tools/gpu_pmc_cls.sh <tag> <cfg> [cfg ...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmcc_$tag
mkdir -p $out
for cfg in "$@"; do
  n=$(echo $cfg | tr ',' '_')
  HRF_CLASSIFY_W16=$cfg timeout -k 10 120 python3 tools/time_classify.py 2 64 256 1023 > $out/scan_$n.txt 2>&1 || exit 1
  cat $out/scan_$n.txt
  HRF_CLASSIFY_W16=$cfg timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/sq1_$n -o pmc -- python3 tools/time_classify.py 2 1023 > $out/sq1_$n.log 2>&1 || exit 1
  HRF_CLASSIFY_W16=$cfg timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE --output-format csv -d $out/sq2_$n -o pmc -- python3 tools/time_classify.py 2 1023 > $out/sq2_$n.log 2>&1 || exit 1
done
python3 tools/pmc_table.py $out

#!/bin/bash
# PMC passes over the exact classifier's kernels (tools/time_classify_exact.py), one counter
# group per rocprofv3 run.  usage: bash tools/gpu_pmc_refine.sh <tag>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_refine_$1
mkdir -p $out
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o pmc -- \
    python3 tools/time_classify_exact.py 3 > $out/$name.log 2>&1
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE &&
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM &&
run tcc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum &&
echo pmc done
python3 - $out <<'PY'
import csv, glob, sys, statistics
out = sys.argv[1]
rows = {}
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "refine" not in k and "w16t" not in k:
            continue
        name = "refine_best" if "refine_best" in k else "refine_list" if "refine_list" in k else "w16t"
        rows.setdefault(name, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for name, cs in rows.items():
    print(name, " ".join("%s=%.4g" % (c, statistics.median(v)) for c, v in sorted(cs.items())))
PY

"""Mean per-dispatch SQ counters of the classify kernels in a gpu_pmc_cls.sh output directory."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
    cfg = os.path.relpath(f, d).split(os.sep)[0].split("_", 1)[1]
    for r in csv.DictReader(open(f)):
        if "classify_pixels" not in r["Kernel_Name"]:
            continue
        rows[cfg][r["Counter_Name"]].append(float(r["Counter_Value"]))
for cfg, c in sorted(rows.items()):
    m = {k: sum(v) / len(v) for k, v in c.items()}
    print("cfg", cfg)
    for k in sorted(m):
        print("  %-28s %16.0f" % (k, m[k]))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        print("  mfma_busy_per_SIMD %.3f" % (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] * 1024 / 8)))
    if "SQ_WAVE_CYCLES" in m:
        t = m["SQ_WAVE_CYCLES"]
        print("  wait_any %.3f wait_inst %.3f active %.3f" % (m["SQ_WAIT_ANY"] / t, m["SQ_WAIT_INST_ANY"] / t,
                                                             m["SQ_ACTIVE_INST_ANY"] / t))

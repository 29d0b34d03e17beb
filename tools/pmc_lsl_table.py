"""Mean per-dispatch SQ counters of the label_sums_lasers kernels in gpu_pmc_lsl.sh's output
directory, per env setting: python tools/pmc_lsl_table.py gpurun_out/pmc_lsl"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
    cfg = os.path.relpath(f, d).split(os.sep)[0].rsplit(".", 1)[0]
    for r in csv.DictReader(open(f)):
        if "label_sums_lasers" not in r["Kernel_Name"]:
            continue
        rows[cfg][r["Counter_Name"]].append(float(r["Counter_Value"]))
for cfg, c in sorted(rows.items()):
    m = {k: sum(v) / len(v) for k, v in c.items()}
    print("cfg", cfg)
    for k in sorted(m):
        print("  %-28s %16.0f" % (k, m[k]))
    if "SQ_WAVE_CYCLES" in m:
        t = m["SQ_WAVE_CYCLES"]
        print("  wait_any %.3f wait_inst %.3f active %.3f" % (m["SQ_WAIT_ANY"] / t, m["SQ_WAIT_INST_ANY"] / t,
                                                             m["SQ_ACTIVE_INST_ANY"] / t))

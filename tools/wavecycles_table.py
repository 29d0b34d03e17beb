"""Per-kernel totals of a rocprofv3 --pmc counter_collection.csv, normalised per tile (the
assemble_ecoli_kernel launch count): SQ_WAVE_CYCLES share = each kernel's part of the wave-slot
time the path occupies.  usage: python tools/wavecycles_table.py <counter_collection.csv>"""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:60]


rows = list(csv.DictReader(open(sys.argv[1])))
tot = collections.defaultdict(lambda: collections.Counter())
disp = collections.defaultdict(set)
for r in rows:
    k = short(r["Kernel_Name"])
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
ntile = max(1, len(disp.get(next((k for k in disp if k.startswith("assemble_ecoli")), ""), ())))
allwc = sum(c["SQ_WAVE_CYCLES"] for c in tot.values())
print("tiles %d; per tile: %-50s %8s %8s %14s %6s %10s %10s %10s" % (ntile, "kernel", "launch", "waves", "wave_cycles", "share",
                                                                   "valu", "salu", "vmem"))
for k, c in sorted(tot.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    print("%-60s %8.1f %8.0f %14.0f %6.3f %10.0f %10.0f %10.0f" % (
        k, len(disp[k]) / ntile, c["SQ_WAVES"] / ntile, c["SQ_WAVE_CYCLES"] / ntile, c["SQ_WAVE_CYCLES"] / allwc,
        c["SQ_INSTS_VALU"] / ntile, c["SQ_INSTS_SALU"] / ntile, c["SQ_INSTS_VMEM"] / ntile))

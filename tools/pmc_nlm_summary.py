"""Summarise tools/gpu_pmc_nlm.sh <tag> (NL-means pair kernel under rocprofv3: kernel trace + two SQ
passes) into profiles/<tag>_nlmeans_pmc.json.

  VALU busy = SQ_INSTS_VALU x 4 cycles (wave64 f64) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)

python tools/pmc_nlm_summary.py <tag> [gpurun_out/pmc_nlm_<tag>]
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = "nl_means_pairs_kernel"


def main():
    tag = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join("gpurun_out", "pmc_nlm_" + tag)
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    durs, name = [], None
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                name = r["Kernel_Name"]
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "sq*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                per[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    c = {k: round(statistics.median(v.values())) for k, v in sorted(per.items())}
    cycles = c["GRBM_GUI_ACTIVE"] / 8
    out = {"round": tag, "kernel": name, "avg_duration_us_kernel_trace": round(statistics.mean(durs), 4),
           "counters_per_dispatch": c,
           "valu_insts_per_simd_cycle": round(c["SQ_INSTS_VALU"] / (cycles * 1024), 4),
           "valu_busy_frac_4cyc": round(4 * c["SQ_INSTS_VALU"] / (cycles * 1024), 4),
           "lds_bank_conflict_frac": round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4),
           "note": "tools/gpu_pmc_nlm.sh over tools/time_kernels.py nlmeans (2048^2); medians per dispatch; "
                   "GRBM_GUI_ACTIVE summed over 8 XCDs; VALU busy = 4 cycles per wave64 f64 instruction"}
    json.dump(out, open(os.path.join(here, "profiles", "%s_nlmeans_pmc.json" % tag), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

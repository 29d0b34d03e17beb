"""Summarise tools/gpu_pmc.sh <tag> t (the isolated pixel-table classifier, R = 1023, under
rocprofv3: kernel trace, FETCH_SIZE, WRITE_SIZE and two SQ passes) into
profiles/classify_pixels_pmc.json (the bench roofline's traffic and counters) and
profiles/<tag>_classify_kernel_stats.csv / <tag>_classify_pmc.json.

  hbm bytes  = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md §HBM: 16-B-per-lane reads, the
               table is read by global_load_lds_dwordx4 / global_load_dwordx4)
  clock      = GRBM_GUI_ACTIVE / 8 XCDs / kernel-trace duration
  mfma busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)  (16 cycles per
               v_mfma_f32_16x16x32_f16)

python tools/pmc_classify_summary.py <tag> [gpurun_out/pmc_<tag>] [kernel substring]
"""
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d, sub):
    vals = {}
    name = None
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                name = r["Kernel_Name"]
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return name, {k: statistics.median(v) for k, v in vals.items()}


def main():
    tag = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "pmc_" + tag)
    sub = sys.argv[3] if len(sys.argv) > 3 else "classify_pixels_w16t_kernel"
    here = os.path.join(REPO, "profiles")
    stats = glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True)
    rows = list(csv.DictReader(open(stats[0])))
    with open(os.path.join(here, "%s_classify_kernel_stats.csv" % tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_us", "pct"])
        for r in rows:
            w.writerow([r["Name"], r["Calls"], "%.3f" % (float(r["TotalDurationNs"]) / 1e6),
                        "%.1f" % (float(r["AverageNs"]) / 1e3), r["Percentage"]])
    st = [r for r in rows if sub in r["Name"]]
    avg_us = float(st[0]["AverageNs"]) / 1e3
    c = {}
    name = None
    for part in ("fetch", "write", "sq1", "sq2"):
        n, v = counters(os.path.join(d, part), sub)
        name = name or n
        c.update(v)
    out = {"kernel": name, "round": tag, "avg_duration_us_kernel_trace": avg_us,
           "fetch_kib_raw": c.get("FETCH_SIZE"), "write_kib": c.get("WRITE_SIZE"),
           "hbm_bytes_per_launch": (c["FETCH_SIZE"] * 2 + c.get("WRITE_SIZE", 0.0)) * 1024 if "FETCH_SIZE" in c else None,
           "counters_median_per_dispatch": c,
           "note": "read side doubled per MI355X_MICROARCH.md §HBM (gfx950 FETCH_SIZE = half of a wide coalesced read); "
                   "counters from separate --pmc passes, medians per dispatch"}
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        out["sclk_mhz_mean"] = round(cyc / avg_us, 1)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            out["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4)
        if "SQ_BUSY_CYCLES" in c:
            out["sq_busy_cycles_per_grbm"] = round(c["SQ_BUSY_CYCLES"] / c["GRBM_GUI_ACTIVE"], 4)
    if "SQ_WAVE_CYCLES" in c:
        t = c["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: round(c[k] / t, 4) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
                                   if k in c}
    json.dump(out, open(os.path.join(here, "classify_pixels_pmc.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(here, "%s_classify_pmc.json" % tag), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

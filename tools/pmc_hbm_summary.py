"""Summarise tools/gpu_pmc_hbm.sh's rocprofv3 outputs into profiles/hbm_kernels_pmc.json (the
bench's hbm_kernels traffic) and profiles/<tag>_hbm_kernel_stats.csv / _pmc_hbm.csv.

Per kernel (bench.py HBM_KERNELS): median per-dispatch FETCH_SIZE and WRITE_SIZE (KiB) from the
separate passes.  Read side: x2 for the 16-byte-per-lane streaming reads (MI355X_MICROARCH.md
§HBM: gfx950 FETCH_SIZE counts half of such reads) -- channel_max_multi_pf (float4 loads) and the
assembly; the lasers label sums read 4 bytes per lane, so their factor is calibrated on the dense
map run (every pixel labelled: algorithmic read bytes known exactly).  WRITE_SIZE as is.

python tools/pmc_hbm_summary.py <tag> [gpurun_out/pmc_hbm]
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import HBM_KERNELS as KERNELS  # noqa: E402  (the kernel symbols live in one place)


def counters(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def pick(vals, sub):
    ks = [k for k in vals if sub in k]
    if not ks:
        return None, None
    return ks[0], statistics.median(vals[ks[0]])


def main():
    tag = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "pmc_hbm")
    stats = glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True)
    rows = list(csv.DictReader(open(stats[0]))) if stats else []
    here = os.path.join(REPO, "profiles")
    with open(os.path.join(here, "%s_hbm_kernel_stats.csv" % tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_us", "pct"])
        for r in rows:
            w.writerow([r["Name"], r["Calls"], "%.3f" % (float(r["TotalDurationNs"]) / 1e6),
                        "%.1f" % (float(r["AverageNs"]) / 1e3), r["Percentage"]])
    alg = {}
    for line in open(os.path.join(d, "kt.log")):
        m = re.match(r"(\w+): ([\d.]+) ms .* (\d+) bytes", line)
        if m:
            alg[m.group(1)] = int(m.group(3))
    fetch, write = counters(os.path.join(d, "fetch"), "FETCH_SIZE"), counters(os.path.join(d, "write"), "WRITE_SIZE")
    cfetch = counters(os.path.join(d, "calfetch"), "FETCH_SIZE")
    # dense calibration: every pixel labelled -> read = label map + 95 channels + flat field per pixel
    H = W = 2048
    dense_read = H * W * (4 + 4 * 95 + 4)
    _, cf = pick(cfetch, KERNELS["label_sums_lasers_cal"])
    lasers_factor = dense_read / (cf * 1024) if cf else None
    out = {"round": tag, "source": "tools/gpu_pmc_hbm.sh (rocprofv3 FETCH_SIZE / WRITE_SIZE passes over "
                                   "tools/time_kernels.py path; calibration over tools/time_kernels.py pathcal)",
           "label_sums_lasers_read_factor": lasers_factor,
           "label_sums_lasers_dense_fetch_kib_raw": cf, "kernels": {}}
    with open(os.path.join(here, "%s_hbm_pmc.csv" % tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["row", "kernel", "FETCH_SIZE_KiB_raw_median", "WRITE_SIZE_KiB_median", "read_factor",
                    "hbm_bytes_per_launch", "algorithmic_bytes", "ratio", "avg_us_kernel_trace"])
        for name, sub in KERNELS.items():
            k, fk = pick(fetch, sub)
            _, wk = pick(write, sub)
            if k is None:
                continue
            factor = lasers_factor if name == "label_sums_lasers_cal" else 2.0
            hbm = fk * 1024 * factor + (wk or 0.0) * 1024
            st = [r for r in rows if sub in r["Name"]]
            avg_us = float(st[0]["AverageNs"]) / 1e3 if st else None
            a = alg.get(name)
            rec = {"kernel": k[:160], "fetch_kib_raw": fk, "write_kib": wk, "read_factor": factor,
                   "hbm_bytes_per_launch": round(hbm), "algorithmic_bytes": a,
                   "traffic_ratio": round(hbm / a, 4) if a else None, "avg_us_kernel_trace": avg_us}
            out["kernels"][name] = rec
            w.writerow([name, k[:90], "%.1f" % fk, "%.1f" % (wk or 0), "%.4f" % factor, "%.0f" % hbm, a,
                        "%.4f" % (hbm / a) if a else "", "%.1f" % avg_us if avg_us else ""])
    json.dump(out, open(os.path.join(here, "hbm_kernels_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

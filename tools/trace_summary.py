"""Per-step kernel summary of a rocprofv3 kernel trace (csv): wall, busy, launches, top kernels,
host-sync gaps.  usage: python tools/trace_summary.py <kernel_trace.csv> <step-marker substring>"""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:60]


def main():
    path, marker = sys.argv[1], sys.argv[2]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[min(2, len(idx) - 2)], idx[-1]
    seg = rows[a:b]
    nst = len([i for i in idx if a <= i < b])
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print("steps %d  wall/step %.3f ms  kernel-busy/step %.3f ms  launches/step %.1f" %
          (nst, (t1 - t0) / nst / 1e6, busy / nst / 1e6, len(seg) / nst))
    d, n = collections.Counter(), collections.Counter()
    for r in seg:
        k = short(r["Kernel_Name"])
        d[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n[k] += 1
    for k, v in d.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30):
        print("%-60s %6.1f/step %8.3f ms/step" % (k, n[k] / nst, v / nst / 1e6))
    # time with no kernel running at all (union of the kernels' intervals; with concurrent
    # streams a gap between two consecutive starts is not idle if a third kernel spans it)
    gap, reach = 0, int(seg[0]["Start_Timestamp"])
    for r in seg:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if a > reach:
            gap += a - reach
        reach = max(reach, b)
    print("idle (no kernel running): %.3f ms/step, %.1f %% of wall" % (gap / nst / 1e6, 100.0 * gap / (t1 - t0)))


if __name__ == "__main__":
    main()

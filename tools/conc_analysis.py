"""Concurrency picture of a rocprofv3 kernel trace of the concurrent bench (csv): per stream the
busy time, the gaps between its consecutive kernels (time its chain waited for the host or a
dependency), and how the wall time splits by what was running (classifier alone, classifier +
other work, other work only, nothing).
usage: python tools/conc_analysis.py <kernel_trace.csv> [classifier substring]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    cls = sys.argv[2] if len(sys.argv) > 2 else "classify_pixels"
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"], r["Queue_Id"])
            for r in csv.DictReader(open(path))]
    rows.sort()
    # keep the steady part: from the 3rd classifier launch to the last one
    cl = [i for i, r in enumerate(rows) if cls in r[2]]
    if len(cl) < 6:
        print("too few classifier launches", len(cl))
        return
    t0, t1 = rows[cl[2]][0], rows[cl[-1]][0]
    rows = [r for r in rows if t0 <= r[0] < t1]
    ntile = len([r for r in rows if cls in r[2]])
    wall = t1 - t0
    # time split by state
    ev = []
    for s, e, n, st, q in rows:
        c = cls in n
        ev.append((s, 1, c))
        ev.append((e, -1, c))
    ev.sort()
    ncl = noth = 0
    last = t0
    acc = collections.Counter()
    for t, d, c in ev:
        t = min(max(t, t0), t1)
        state = ("cls" if ncl else "") + ("+oth" if noth else "")
        acc[state or "idle"] += t - last
        last = t
        if c:
            ncl += d
        else:
            noth += d
    print("tiles (classifier launches) %d, wall %.3f ms, %.3f ms per tile" % (ntile, wall / 1e6, wall / 1e6 / ntile))
    for k, v in acc.most_common():
        print("  %-10s %6.1f %%  %.3f ms per tile" % (k, 100 * v / wall, v / 1e6 / ntile))
    # per stream: busy, gaps
    by = collections.defaultdict(list)
    for r in rows:
        by[r[3]].append(r)
    print("per stream (launches, busy ms per tile, gap ms per tile, share of classifier launches):")
    for st, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
        rs.sort()
        busy = sum(e - s for s, e, *_ in rs)
        gap = 0
        reach = rs[0][1]
        for s, e, *_ in rs[1:]:
            if s > reach:
                gap += s - reach
            reach = max(reach, e)
        nc = sum(cls in r[2] for r in rs)
        print("  stream %-4s %6d  busy %.3f  gaps %.3f  classifier %d" % (st, len(rs), busy / 1e6 / ntile, gap / 1e6 / ntile, nc))


if __name__ == "__main__":
    main()

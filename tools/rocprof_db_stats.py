"""Per-kernel summary of a rocprofv3 --kernel-trace run (run_results.db, sqlite `kernels`
table): calls, total / mean duration, share of the summed kernel time.

python tools/rocprof_db_stats.py RUN_RESULTS.DB [OUT.csv] [TOP]
"""
import csv
import re
import sqlite3
import sys


def rows(db):
    c = sqlite3.connect(db)
    out = list(c.execute("select name, count(*), sum(end-start) from kernels group by name order by sum(end-start) desc"))
    return out


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:100]


def main():
    db = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2].endswith(".csv") else None
    top = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 30
    rs = rows(db)
    tot = sum(r[2] for r in rs)
    print("summed kernel time %.2f ms" % (tot / 1e6))
    for n, calls, td in rs[:top]:
        print("%9.2f ms %7d %10.1f us %5.1f%%  %s" % (td / 1e6, calls, td / calls / 1e3, 100.0 * td / tot, short(n)))
    if out:
        with open(out, "w") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "total_ms", "avg_us", "pct"])
            for n, calls, td in rs:
                w.writerow([short(n), calls, "%.3f" % (td / 1e6), "%.1f" % (td / calls / 1e3), "%.2f" % (100.0 * td / tot)])


if __name__ == "__main__":
    main()

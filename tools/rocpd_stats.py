"""Per-kernel summary of a rocprofv3 SQLite output (``-o run`` writes run_results.db on this ROCm):
kernel name, calls, total / average / min / max duration (us), share of the total, sorted by total time.

    python tools/rocpd_stats.py <run_results.db> [--csv out.csv] [--match REGEX]
"""
import argparse
import csv
import re
import sqlite3


def stats(db, match=None):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute("select %s, start, end from kernels" % name_col).fetchall()
    agg = {}
    for n, s, e in rows:
        if match and not re.search(match, n):
            continue
        a = agg.setdefault(n, [0, 0.0, float("inf"), 0.0])
        d = (e - s) / 1e3
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(v[1] for v in agg.values()) or 1.0
    out = [(n, v[0], v[1], v[1] / v[0], v[2], v[3], 100 * v[1] / tot) for n, v in agg.items()]
    out.sort(key=lambda r: -r[2])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--match", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    out = stats(a.db, a.match)
    for n, calls, tot, avg, mn, mx, pct in out[:a.top]:
        print("%10.1f us %6d calls %10.2f avg %6.2f%%  %s" % (tot, calls, avg, pct, n[:110]))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "MinUs", "MaxUs", "Percentage"])
            for r in out:
                w.writerow([r[0], r[1], "%.3f" % r[2], "%.3f" % r[3], "%.3f" % r[4], "%.3f" % r[5], "%.2f" % r[6]])


if __name__ == "__main__":
    main()

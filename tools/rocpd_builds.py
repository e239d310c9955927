"""Per-call breakdown of repeated tagan_csr_build calls in a rocprofv3 SQLite output: the kernels between two
k_init launches form one build; prints every ``--every``-th build's kernels (us).

    python tools/rocpd_builds.py <run_results.db> [--every 5] [--first-kernel k_init]
"""
import argparse
import collections
import re
import sqlite3


def short(n):
    n = n.replace("(anonymous namespace)", "anon").replace("void ", "")
    n = n.split("(")[0]
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--every", type=int, default=5)
    ap.add_argument("--first-kernel", default="k_init")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    builds, cur = [], None
    for n, s, e in rows:
        sn = short(n)
        if sn == a.first_kernel:
            cur = []
            builds.append(cur)
        if cur is not None and "tagan" in n:
            cur.append((sn, (e - s) / 1e3))
    for bi, b in enumerate(builds):
        if bi % a.every != a.every - 1:
            continue
        agg = collections.OrderedDict()
        for n, d in b:
            agg[n] = agg.get(n, 0) + d
        print("build %d: %.1f us device" % (bi, sum(agg.values())))
        for n, d in agg.items():
            print("   %-28s %9.1f" % (n, d))


if __name__ == "__main__":
    main()

"""Per-kernel PMC counter totals from one or more rocprofv3 --pmc SQLite outputs.

    python tools/rocpd_pmc.py gpurun_out/x/p1/run_results.db [more.db ...] [--filter csr] [--per-dispatch]

Prints one row per kernel (short name): dispatches, summed duration (us) and each counter summed over the
kernel's dispatches (or averaged per dispatch with --per-dispatch)."""
import argparse
import collections
import sqlite3


def short(name):
    n = name.replace("(anonymous namespace)", "anon")
    n = n.split("(")[0]
    return n.split("::")[-1][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--per-dispatch", action="store_true")
    a = ap.parse_args()
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    cols = []
    for db in a.dbs:
        c = sqlite3.connect(db)
        for name, did, d, cn, cv in c.execute(
                "select name, dispatch_id, duration, counter_name, counter_value from pmc_events"):
            k = short(name)
            if a.filter and a.filter not in name:
                continue
            rows[k][cn] += cv
            disp[k].add((db, did))
            dur[k][(db, did)] = d
            if cn not in cols:
                cols.append(cn)
    print("%-40s %5s %10s " % ("kernel", "n", "dur_us") + " ".join("%14s" % x[:14] for x in cols))
    for k in sorted(rows, key=lambda k: -sum(dur[k].values())):
        n = len({d for _, d in disp[k]}) or 1
        f = 1.0 / n if a.per_dispatch else 1.0
        print("%-40s %5d %10.1f " % (k, n, sum(dur[k].values()) / 1e3 * f)
              + " ".join("%14.4g" % (rows[k].get(x, 0) * f) for x in cols))


if __name__ == "__main__":
    main()

"""Median per-dispatch value of every PMC counter per kernel under a rocprofv3 output tree.

    python tools/pmc_table.py gpurun_out/sq_<tag> [kernel-substring]
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if filt not in name:
                continue
            short = re.sub(r"^void |tagan::|\(anonymous namespace\)::", "", name)
            short = re.sub(r"\(.*", "", short)[:70]
            vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        print(k)
        for c, v in sorted(cs.items()):
            v = sorted(v)
            print("   %-26s %16.0f  (n=%d)" % (c, v[len(v) // 2], len(v)))


if __name__ == "__main__":
    main()

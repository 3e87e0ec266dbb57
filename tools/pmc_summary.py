"""Sum rocprofv3 --pmc counter_collection.csv rows per (kernel, counter) and print one
line per kernel whose name matches a filter (kernel names shortened).

usage: python tools/pmc_summary.py <counter_collection.csv> [name-substring]
"""
from __future__ import annotations

import collections
import csv
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        if filt and filt not in name:
            continue
        short = name.replace("(anonymous namespace)::", "").split("(")[0][-60:]
        sums[short][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[short].add(row["Dispatch_Id"])
    for k, c in sums.items():
        n = len(disp[k])
        print(k, f"dispatches={n}", " ".join(f"{a}={v / n:.4g}" for a, v in sorted(c.items())))


if __name__ == "__main__":
    main()

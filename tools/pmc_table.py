#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection.csv files: per kernel, per
counter, summed over dispatches (and XCD/SE instances)."""
import csv
import sys
from collections import defaultdict


def main(paths):
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in paths:
        with open(p) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].replace("okm::", "")
                agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(name, r["Counter_Name"])].add(r["Dispatch_Id"])
    for k in sorted(agg):
        print(k)
        for c, v in sorted(agg[k].items()):
            nd = len(disp[(k, c)])
            print(f"   {c:<26} {v:>18.0f}   per-dispatch {v / max(nd, 1):>16.0f}  ({nd} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1:])

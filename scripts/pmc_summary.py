"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel name, mean counter value per dispatch."""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: defaultdict(list))
    for r in rows:
        name = r.get("Kernel_Name") or r.get("Kernel-Name")
        agg[name][r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    return agg


def main(paths):
    merged = defaultdict(dict)
    for p in paths:
        for k, cs in load(p).items():
            for c, vals in cs.items():
                # sum over per-XCD/SE instances of one dispatch, then average over dispatches
                per = defaultdict(float)
                for d, v in vals:
                    per[d] += v
                merged[k][c] = sum(per.values()) / len(per)
    for k, cs in merged.items():
        short = k.split("(")[0][-60:]
        print(short)
        for c in sorted(cs):
            print(f"   {c:32s} {cs[c]:.4g}")


if __name__ == "__main__":
    main(sys.argv[1:])

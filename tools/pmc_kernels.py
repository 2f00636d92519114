"""Summarise rocprofv3 --pmc counter CSVs per kernel (median over dispatches).

Usage: python tools/pmc_kernels.py <counter_collection.csv> [name-substring ...]
Prints, per kernel whose name matches, the median of every collected counter
over its dispatches (rocprofv3 reports one row per dispatch and counter)."""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    pats = sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(dict))
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
        if pats and not any(p in name for p in pats):
            continue
        disp = row.get("Dispatch_Id") or row.get("Dispatch-Id")
        cn = row.get("Counter_Name") or row.get("Counter-Name")
        cv = float(row.get("Counter_Value") or row.get("Counter-Value"))
        vals[name[:80]][cn][disp] = vals[name[:80]][cn].get(disp, 0.0) + cv
    for name, counters in vals.items():
        print(name)
        for cn, per in sorted(counters.items()):
            print(f"  {cn:32s} {statistics.median(per.values()):16.0f}  (n={len(per)})")


if __name__ == "__main__":
    main()

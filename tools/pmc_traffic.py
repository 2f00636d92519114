"""Summarise rocprofv3 PMC passes into HBM traffic per launch of one kernel.

Usage (after two separate `rocprofv3 --pmc FETCH_SIZE ...` / `--pmc WRITE_SIZE ...`
runs with --output-format csv):
    python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <out.json> [alg_bytes]
Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B streaming stores.
"""
import csv
import glob
import json
import os
import statistics
import sys


def counter_values(d, counter, kernel_sub):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if kernel_sub in name and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fd, wd, ksub, out = sys.argv[1:5]
    alg = float(sys.argv[5]) if len(sys.argv) > 5 else None
    fetch = counter_values(fd, "FETCH_SIZE", ksub)
    write = counter_values(wd, "WRITE_SIZE", ksub)
    if not fetch or not write:
        raise SystemExit(f"no samples for {ksub}: fetch {len(fetch)} write {len(write)}")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    traffic = (2.0 * f_kib + w_kib) * 1024.0
    res = {"kernel": ksub, "launches": [len(fetch), len(write)],
           "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib,
           "read_bytes_corrected": 2.0 * f_kib * 1024.0, "write_bytes": w_kib * 1024.0,
           "traffic_bytes_per_launch": traffic, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": (traffic / alg) if alg else None,
           "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KiB -> bytes"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

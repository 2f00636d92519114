"""Summarise rocprofv3 --pmc counter CSVs per kernel (median over dispatches).

Usage: python tools/pmc_kernels.py <counter_collection.csv or glob> [name-substring ...]
       python tools/pmc_kernels.py --filter <rocprofv3 output dir> name-substring ...
Several passes (one CSV each, e.g. "out/mode_p*/run_counter_collection.csv")
are merged per kernel name.  Prints, per kernel whose name matches, the median
of every collected counter over its dispatches and the derived figures the
MI355X_MICROARCH.md guide prescribes:
  HBM bytes = 2 x FETCH_SIZE (gfx950 halves wide streaming reads) + WRITE_SIZE, KiB -> B;
  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY count quad-cycles, split of wave time;
  effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time."""
import collections
import csv
import glob
import statistics
import sys


def load(paths, pats):
    vals = collections.defaultdict(lambda: collections.defaultdict(dict))
    meta = {}
    for path in paths:
        for row in csv.DictReader(open(path)):
            name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
            if pats and not any(p in name for p in pats):
                continue
            key = name[:90]
            disp = (path, row.get("Dispatch_Id") or row.get("Dispatch-Id"))
            cn = row.get("Counter_Name") or row.get("Counter-Name")
            cv = float(row.get("Counter_Value") or row.get("Counter-Value"))
            vals[key][cn][disp] = vals[key][cn].get(disp, 0.0) + cv
            try:
                dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
                vals[key]["_wall_s"][disp] = dur
            except (KeyError, ValueError):
                pass
            meta[key] = {k: row.get(k) for k in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size",
                                                 "Scratch_Size", "Grid_Size", "Workgroup_Size")}
    return vals, meta


def filter_dir(d, pats):
    """Keep only the rows of kernels matching pats in d's counter CSVs and drop
    every other rocprofv3 output file (keeps gpurun_out/ small)."""
    import os
    for root, _, files in os.walk(d):
        for f in files:
            path = os.path.join(root, f)
            if not f.endswith("counter_collection.csv"):
                os.remove(path)
                continue
            with open(path) as fh:
                rows = list(csv.reader(fh))
            head, body = rows[0], rows[1:]
            ki = head.index("Kernel_Name")
            with open(path, "w", newline="") as fh:
                w = csv.writer(fh, quoting=csv.QUOTE_MINIMAL)
                w.writerow(head)
                w.writerows(r for r in body if any(p in r[ki] for p in pats))


def main():
    if sys.argv[1] == "--filter":
        filter_dir(sys.argv[2], sys.argv[3:])
        return
    paths = []
    for a in sys.argv[1:2]:
        paths += sorted(glob.glob(a)) if any(c in a for c in "*?[") else [a]
    pats = sys.argv[2:]
    vals, meta = load(paths, pats)
    for name, counters in vals.items():
        med = {cn: statistics.median(per.values()) for cn, per in counters.items()}
        print(name)
        print("  " + " ".join(f"{k}={v}" for k, v in meta[name].items()))
        for cn in sorted(med):
            if cn.startswith("_"):
                continue
            print(f"  {cn:32s} {med[cn]:18.1f}  (n={len(counters[cn])})")
        wall = med.get("_wall_s")
        if wall:
            print(f"  {'wall_us (profiled, median)':32s} {wall * 1e6:18.1f}")
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            rd, wr = 2.0 * med["FETCH_SIZE"] * 1024.0, med["WRITE_SIZE"] * 1024.0
            print(f"  HBM read (2 x FETCH_SIZE) {rd / 1e6:12.2f} MB   write {wr / 1e6:10.2f} MB   total {(rd + wr) / 1e6:10.2f} MB")
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            parts = {k: med.get(k) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
            print("  wave-cycle split: " + ", ".join(f"{k[3:]} {v / wc:.3f}" for k, v in parts.items() if v is not None))
        waves = med.get("SQ_WAVES")
        if waves:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_VMEM_WR"):
                if k in med:
                    print(f"  {k + ' per wave':32s} {med[k] / waves:18.1f}")
        if "SQ_LDS_BANK_CONFLICT" in med and med.get("SQ_LDS_IDX_ACTIVE"):
            print(f"  LDS bank-conflict share {med['SQ_LDS_BANK_CONFLICT'] / med['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "GRBM_GUI_ACTIVE" in med and wall:
            print(f"  effective clock {med['GRBM_GUI_ACTIVE'] / 8 / wall / 1e9:.2f} GHz (GRBM_GUI_ACTIVE / 8 / wall)")


if __name__ == "__main__":
    main()

"""Text summary of a rocprofv3 --kernel-trace --stats run (run_kernel_stats.csv).

Usage: python tools/prof_summary.py <run_kernel_stats.csv> "<header line>" > profiles/<tag>_rocprof_stats.txt
Columns: kernel (truncated), calls, average / min / max duration in us, share of
the total kernel time, sorted by total time."""
import csv
import sys


def main():
    path, header = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    rows = []
    for r in csv.DictReader(open(path)):
        name = r.get("Name") or r.get("Kernel_Name") or ""
        rows.append((name, int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
                     float(r["MaxNs"]) / 1e3, float(r["Percentage"])))
    rows.sort(key=lambda t: -t[5])
    if header:
        print(header)
    print(f"{'kernel':72s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'pct':>6s}")
    for name, calls, avg, mn, mx, pct in rows:
        print(f"{name[:72]:72s} {calls:6d} {avg:10.1f} {mn:10.1f} {mx:10.1f} {pct:6.2f}")


if __name__ == "__main__":
    main()

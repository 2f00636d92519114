"""Checks one bench.py JSON line (a file holding it) for the contract fields:
nodes_total = 8 (configs[2]), roofline, cpu_baseline, an xgmi block at N > 1,
and no errored extra.  Prints a one-line summary; exit 1 on a failed check.
Usage: python tools/check_bench_line.py <line.json> <N>"""
import json
import sys


def check(line, n):
    bad = []
    if line.get("n_gpus") != n:
        bad.append(f"n_gpus {line.get('n_gpus')} != {n}")
    if line.get("config", {}).get("nodes_total") != 8:
        bad.append(f"nodes_total {line.get('config', {}).get('nodes_total')} != 8")
    if not line.get("roofline"):
        bad.append("no roofline")
    if not line.get("cpu_baseline"):
        bad.append("no cpu_baseline")
    if n > 1 and not line.get("xgmi"):
        bad.append("no xgmi block")
    for k, v in (line.get("extras") or {}).items():
        if isinstance(v, dict) and "error" in v:
            bad.append(f"extra {k}: {v['error']}")
    return bad


if __name__ == "__main__":
    text = open(sys.argv[1]).read().strip().splitlines()
    line = json.loads([t for t in text if t.startswith("{")][-1])
    bad = check(line, int(sys.argv[2]))
    print(f"n_gpus {line.get('n_gpus')} nodes_total {line.get('config', {}).get('nodes_total')} "
          f"value {line.get('value')} ms {line.get('ms_per_step')} frac {line.get('roofline', {}).get('frac')} "
          f"cpu {(line.get('cpu_baseline') or {}).get('value')} extras "
          f"{ {k: (v.get('ms_per_step') if isinstance(v, dict) else v) for k, v in (line.get('extras') or {}).items()} }")
    for b in bad:
        print("FAIL:", b)
    sys.exit(1 if bad else 0)

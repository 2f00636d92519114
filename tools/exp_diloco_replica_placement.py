"""The headline DiLoCo step across fresh processes with and without the replica-set
stage of DiLoCoOuter's placement (engine.REPLICA_PLACEMENT_CANDIDATES; diagnostic,
round 5).  The parent never touches the GPU: it starts `python tools/exp_diloco_
replica_placement.py --child on|off` processes alternately; each child sets the
constant (off: 0) and runs bench.py's main (--no-extras --no-cpu-baseline --no-pmc),
and the parent prints one JSON line per child: kernel ms, frac, the replica-set and
master probe minima.  Usage: python tools/exp_diloco_replica_placement.py [pairs] [modes: on,off or e.g. on,20]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode):
    sys.path.insert(0, ROOT)
    from gym_amd import engine
    if mode == "off":
        engine.REPLICA_PLACEMENT_CANDIDATES = 0
    elif mode.isdigit():  # a candidate count other than the default
        engine.REPLICA_PLACEMENT_CANDIDATES = int(mode)
    import bench
    sys.argv = ["bench.py", "--no-extras", "--no-cpu-baseline", "--no-pmc", "--steps", "20", "--warmup", "3"]
    bench.main()


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["on", "off"]
    for i in range(pairs):
        for mode in modes:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode], capture_output=True,
                               text=True, timeout=300, cwd=ROOT)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not lines:
                print(json.dumps({"mode": mode, "error": r.stderr[-500:]}), flush=True)
                sys.exit(1)
            d = json.loads(lines[-1])
            rf = d["roofline"]
            pl = rf.get("placement") or {}
            rep = pl.get("replica_set") or {}
            print(json.dumps({"pair": i, "mode": mode, "kernel_ms": rf["kernel_ms"], "frac": rf["frac"],
                              "replica_probe_min": min(rep["probe_ms"]) if rep.get("probe_ms") else None,
                              "replica_probe_own": rep["probe_ms"][0] if rep.get("probe_ms") else None,
                              "replica_chosen": rep.get("chosen"),
                              "master_probe_min": min(pl["probe_ms"]) if pl.get("probe_ms") else None}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()

"""Flag `file.py:LINE[-LINE]` citations that point past the end of the cited
reference file (exogym/... under /root/reference).  Run in the build
container only (the reference is not on the GPU box).

usage: python tools/check_citations.py [paths...]
"""
import os
import re
import sys

REF = "/root/reference"
PAT = re.compile(r"((?:[\w./]+/)?[\w]+\.py):(\d+)(?:-(\d+))?")


def ref_files():
    out = {}
    for d, _, fs in os.walk(REF):
        for f in fs:
            if f.endswith(".py"):
                p = os.path.join(d, f)
                rel = os.path.relpath(p, REF)
                out.setdefault(f, []).append((rel, sum(1 for _ in open(p, errors="replace"))))
    return out


def main(paths):
    files = ref_files()
    bad = 0
    for root in paths:
        walk = [(root, None, [root])] if os.path.isfile(root) else os.walk(root)
        for d, _, fs in walk:
            for f in fs:
                p = f if d == root and os.path.isfile(root) else os.path.join(d, f)
                if not p.endswith((".py", ".h", ".hip", ".md")) or "/golden/" in p and p.endswith(".npz"):
                    continue
                for ln, line in enumerate(open(p, errors="replace"), 1):
                    for m in PAT.finditer(line):
                        name = os.path.basename(m.group(1))
                        cands = files.get(name)
                        if not cands:
                            continue
                        if "/" in m.group(1):
                            cands = [c for c in cands if c[0].endswith(m.group(1))] or cands
                        hi = int(m.group(3) or m.group(2))
                        if all(hi > n for _, n in cands):
                            print(f"{p}:{ln}: {m.group(0)} past the end of {[c[0] for c in cands]} "
                                  f"({[n for _, n in cands]} lines)")
                            bad += 1
    return bad


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1:] or ["gym_amd", "include", "oracle", "tests", "exogym", "INTEGRATION.md",
                                         "DESIGN.md", "bench.py", "__graft_entry__.py"]) else 0)

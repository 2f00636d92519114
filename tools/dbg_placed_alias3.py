"""Debug aid (not part of the library; round 5): the r04u
corruption of a kept PlacedBuffer (hipMemCreate + hipMemAddressReserve + map)
when ordinary torch allocations are made between creations -- do the placed
virtual ranges overlap the caching allocator's segments?  Repeats the
dbg_placed_alias.py pattern (create + fill buffer i, then check buffer 0 with
torch temporaries) and after every step compares every placed range
[va, va + nbytes) with every segment of torch.cuda.memory_snapshot()
(address, total_size), and reports the first corruption together with any
overlap."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from placed_buffer import PlacedBuffer  # noqa: E402

DEV = torch.device("cuda:0")


def segments():
    return [(s["address"], s["address"] + s["total_size"], s.get("segment_type", "?"))
            for s in torch.cuda.memory_snapshot() if s.get("device", 0) == 0]


def overlaps(bufs, segs):
    out = []
    for i, b in enumerate(bufs):
        a0, a1 = b.va.value, b.va.value + b.nbytes
        for s0, s1, kind in segs:
            if s0 < a1 and a0 < s1:
                out.append((i, hex(a0), hex(a1), hex(s0), hex(s1), kind))
    return out


def trial(nbytes, ncand):
    bufs, first_bad = [], None
    for i in range(ncand):
        b = PlacedBuffer(nbytes, DEV)
        b.tensor(torch.uint8).fill_(i + 1)
        torch.cuda.synchronize()
        bufs.append(b)
        bad0 = int((bufs[0].tensor(torch.uint8) != 1).sum())  # torch temporaries: a bool tensor + a sum
        ov = overlaps(bufs, segments())
        print(f"  after #{i}: buffer 0 changed bytes {bad0}; placed/segment overlaps {len(ov)} {ov[:3]}", flush=True)
        if bad0 and first_bad is None:
            first_bad = i
    vas = [(hex(b.va.value), b.nbytes) for b in bufs]
    segs = [(hex(a), b - a, k) for a, b, k in segments()]
    print(f"  placed ranges {vas[:4]} ...; torch segments {segs[:6]}", flush=True)
    torch.cuda.synchronize()
    for b in bufs:
        b.release()
    return first_bad


def main():
    for nbytes in (50331648, 1_400_000_000):
        print(f"{nbytes} B x 16: first corruption at creation #{trial(nbytes, 16)}", flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

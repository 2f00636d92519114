"""Debug aid (not part of the library): does a kept PlacedBuffer stay intact when
the other physical allocations created around it are released and ordinary torch
allocations are then made and written?  Sizes as the DeMo test (48 MiB) and as
the DiLoCo / 350M buffers (1.4 GiB)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from placed_buffer import PlacedBuffer  # noqa: E402

DEV = torch.device("cuda:0")


def trial(nbytes, ncand, keep_idx):
    bufs = []
    for i in range(ncand):
        b = PlacedBuffer(nbytes, DEV)
        b.tensor(torch.uint8).fill_(i + 1)
        torch.cuda.synchronize()
        bad0 = int((bufs[0].tensor(torch.uint8) != 1).sum()) if bufs else 0
        if bad0:
            print(f"   after creating+filling #{i}: buffer 0 has {bad0} changed bytes", flush=True)
        bufs.append(b)
    vas = sorted((b.va.value, b.va.value + b.nbytes, i) for i, b in enumerate(bufs))
    overl = [(a[2], c[2]) for a, c in zip(vas, vas[1:]) if c[0] < a[1]]
    keep = bufs[keep_idx]
    torch.cuda.synchronize()
    for i, b in enumerate(bufs):
        if i != keep_idx:
            b.release()
    t = keep.tensor(torch.uint8)
    ok0 = bool((t == keep_idx + 1).all())
    junk = [torch.full((nbytes // 4,), 77, dtype=torch.int32, device=DEV) for _ in range(2 * ncand)]
    torch.cuda.synchronize()
    ok1 = bool((t == keep_idx + 1).all())
    bad = int((t != keep_idx + 1).sum())
    del junk
    keep.release()
    return ok0, ok1, bad, "VA overlaps", overl


def main():
    for nbytes in (50356224, 48 << 20, 1_400_000_000):
        for keep_idx in (0, 5, 15):
            print(f"{nbytes} B x 16, keep #{keep_idx}: intact after releases / after torch writes / bad bytes",
                  trial(nbytes, 16, keep_idx), flush=True)


if __name__ == "__main__":
    main()

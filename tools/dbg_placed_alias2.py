"""Debug aid (not part of the library): is the corruption of a PlacedBuffer seen
by dbg_placed_alias.py aliasing between VMM allocations, or between a VMM
allocation and ordinary (caching-allocator) memory?  (A) 16 buffers created and
filled with no torch allocation in between, checked into preallocated outputs;
(B) then ordinary torch allocations made and written, buffers checked again."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from placed_buffer import PlacedBuffer  # noqa: E402

DEV = torch.device("cuda:0")


def main():
    for nbytes in (48 << 20, 1 << 30):
        n = nbytes
        neq = torch.empty(n, dtype=torch.bool, device=DEV)
        cnt = torch.empty((), dtype=torch.int64, device=DEV)

        def bad(b, v):
            torch.ne(b.tensor(torch.uint8)[:n], v, out=neq)
            torch.sum(neq, dim=(0,), out=cnt)
            return int(cnt)
        bufs = []
        for i in range(16):
            b = PlacedBuffer(nbytes, DEV)
            b.tensor(torch.uint8).fill_(i + 1)
            bufs.append(b)
        torch.cuda.synchronize()
        print(f"{nbytes} B: (A) bad bytes per buffer after creating+filling all:",
              [bad(b, i + 1) for i, b in enumerate(bufs)], flush=True)
        junk = [torch.full((nbytes // 4,), 0x4D4D4D4D, dtype=torch.int32, device=DEV) for _ in range(24)]
        torch.cuda.synchronize()
        print(f"{nbytes} B: (B) after 24 ordinary allocations written:",
              [bad(b, i + 1) for i, b in enumerate(bufs)], flush=True)
        del junk
        for b in bufs[1:]:
            b.release()
        junk = [torch.full((nbytes // 4,), 0x4D4D4D4D, dtype=torch.int32, device=DEV) for _ in range(24)]
        torch.cuda.synchronize()
        print(f"{nbytes} B: (C) buffer 0 after releasing the others and 24 more ordinary allocations:",
              bad(bufs[0], 1), flush=True)
        del junk
        bufs[0].release()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

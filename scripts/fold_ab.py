"""A/B of the streaming fold's chunk length / prefetch depth (FLTEE_FOLD_CLOG,
FLTEE_FOLD_DEPTH, read once per process: one process per setting).  C5-shaped input:
M = 2^27 sorted records (1000 x 100K client records + the 10M initial entries + pads),
halo n = 1000.  Prints one JSON line: the setting, us per fold, a checksum of the output
(must agree across settings)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fl-tee_amd"))
from fltee import device as D  # noqa: E402

CASES = {"c5": (1000, 10_000_000, 100_000), "c3": (100, 50890, 5089)}


def main():
    n, d, k = CASES[sys.argv[1] if len(sys.argv) > 1 else "c5"]
    nrec, L = n * k, n * k + d
    M = 1 << (L - 1).bit_length()
    g = torch.Generator(device="cuda").manual_seed(5)
    idx = torch.cat([torch.randint(0, d, (nrec,), generator=g, device="cuda"),
                     torch.arange(d, device="cuda"),
                     torch.full((M - L,), 0xFFFFFFFF, dtype=torch.int64, device="cuda")])
    idx, _ = torch.sort(idx)
    vb = torch.randint(0, 1 << 30, (M,), generator=g, device="cuda")
    src = (idx | (vb << 32)).contiguous()
    del idx, vb
    dst = torch.empty_like(src)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(3):
        D.fold(src, dst, L, n, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        D.fold(src, dst, L, n, st)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    chk = int((dst & 0xFFFFFFFFFFFF).sum().item())
    print(json.dumps(dict(case=sys.argv[1] if len(sys.argv) > 1 else "c5", M=M,
                          clog=os.environ.get("FLTEE_FOLD_CLOG", "auto"),
                          depth=os.environ.get("FLTEE_FOLD_DEPTH", "auto"),
                          us=round(us, 1), status=int(st.item()), chk=chk)), flush=True)


if __name__ == "__main__":
    main()

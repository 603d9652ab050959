"""Debug aid: hashes of the bitonic network output per (mode, m, stages) so two runs
(FLTEE_BITONIC_DIRECT=1 / 0) can be compared.  python scripts/debug_direct.py OUT.json"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))


def main():
    import torch
    from fltee import _lib as L
    from fltee import device as D
    lib = L.lib()
    out = {}
    for mlog in (16, 20, 22):
        m = 1 << mlog
        g = torch.Generator(device="cuda").manual_seed(mlog)
        base = torch.randint(0, 1 << 20, (m,), generator=g, device="cuda", dtype=torch.int64)
        base = base | (torch.arange(m, device="cuda", dtype=torch.int64) << 32)
        for mode in (0, 2):
            for slog in range(12, mlog + 1):
                x = base.clone()
                # stages 1..slog only (segment sort) via the range API on the whole array
                st = lib.fltee_bitonic_range_sort_device(ctypes.c_void_p(x.data_ptr()), 1 << slog, 0, mode, 7, None) if slog == mlog else None
                if slog < mlog:
                    for r in range(m >> slog):
                        seg = x[r << slog:(r + 1) << slog]
                        D.bitonic_range_sort(seg, r << slog, mode=mode, seed=7)
                torch.cuda.synchronize()
                out[f"{mode}/{mlog}/{slog}"] = hashlib.sha1(x.cpu().numpy().tobytes()).hexdigest()[:12]
    json.dump(out, open(sys.argv[1], "w"), indent=0)


if __name__ == "__main__":
    main()

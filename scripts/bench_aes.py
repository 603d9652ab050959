#!/usr/bin/env python3
"""Timing of the AES-128-CTR decrypt kernel (bitsliced, constant time; the library has
no other variant since round 3 — the round-2 A/B against the T-table kernel is in
profiles/r02/ab/aes_variants.jsonl).  Prints one JSON line per shape: kernel ms (HIP events around one decrypt call,
best of K) and GB/s of ciphertext read + records written."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))


def main():
    import torch
    from fltee import device as D
    variant = "bitsliced4"
    shapes = [("ns 100 x 1M dense", 100, 1_000_000), ("c3 100 x 5089 sparse", 100, 5089),
              ("c5 1000 x 100K sparse", 1000, 100_000)]
    for name, n, rpc in shapes:
        ids = np.arange(n, dtype=np.uint32) + 1
        rec = torch.randint(-2**62, 2**62, (n * rpc,), dtype=torch.int64, device="cuda")
        cipher = torch.empty_like(rec)
        D.decrypt(ids, rec, rpc * 8, cipher)
        plain = torch.empty_like(rec)
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            D.decrypt(ids, cipher, rpc * 8, plain)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        assert torch.equal(plain, rec)
        t = min(ts) / 1e3
        print(json.dumps(dict(variant=variant, shape=name, bytes=n * rpc * 8, ms=t * 1e3,
                              gbs=2 * n * rpc * 8 / t / 1e9)), flush=True)
        del rec, cipher, plain
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

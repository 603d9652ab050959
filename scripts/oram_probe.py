"""Time the tree Path ORAM (k_oram.hip) on one exp5 shape, for rocprofv3 / A/B:
    python scripts/oram_probe.py [n] [k] [d]"""
import sys
import time

import torch

sys.path[:0] = [".", "fl-tee_amd"]
from fltee import device as D  # noqa: E402

n, k, d = (int(x) for x in (sys.argv[1:4] + ["3", "5089", "50890"][len(sys.argv) - 1:]))
g = torch.Generator(device="cuda").manual_seed(1)
idx = torch.argsort(torch.rand(n, d, generator=g, device="cuda"), dim=1)[:, :k].to(torch.int64)
vals = torch.randn(n, k, generator=g, device="cuda") * 0.01
rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
out = torch.empty(d, dtype=torch.float32, device="cuda")
for lazy in (False, True):
    A = n * k if lazy else 2 * n * k + 2 * d  # oram.rs's sequence: d + 2 n k + d accesses
    for r in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.aggregate(5, rec, n, k, d, out=out, oram_tree=True, oram_lazy=lazy, seed=3 + r)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        print(f"{'lazy' if lazy else 'ref '} n={n} k={k} d={d}: {A} accesses, {t * 1e3:.2f} ms, "
              f"{t * 1e6 / A:.3f} us/access", flush=True)
assert D.status() == 0

"""H2D of a small ECALL payload, three ways (VERDICT r4 item 4's staging question): a host
memcpy into pinned memory + one DMA, one DMA straight from pageable memory (the runtime
stages it), and the host memcpy alone.  Sizes 12 KB - 12 MB, best of 20, µs.
    python scripts/h2d_probe.py"""
import json
import time

import numpy as np
import torch

dev = torch.device("cuda", 0)
for nbytes in (12 << 10, 122 << 10, 1221 << 10, 4 << 20, 12 << 20):
    src = np.random.default_rng(1).integers(0, 255, nbytes, dtype=np.uint8)
    pinned = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    pn = pinned.numpy()
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    res = {"bytes": nbytes}
    for name in ("memcpy_only", "memcpy_pinned_dma", "pageable_dma"):
        best = 1e9
        for _ in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if name == "memcpy_only":
                np.copyto(pn, src)
            elif name == "memcpy_pinned_dma":
                np.copyto(pn, src)
                with torch.cuda.stream(s):
                    dst.copy_(pinned, non_blocking=True)
                s.synchronize()
            else:
                with torch.cuda.stream(s):
                    dst.copy_(torch.from_numpy(src), non_blocking=False)
                s.synchronize()
            best = min(best, time.perf_counter() - t0)
        res[name + "_us"] = round(best * 1e6, 2)
    print(json.dumps(res), flush=True)

"""A/B in one process: the networks with and without the pad-only stage-block skip
(fltee_debug_set_pad_skip) at configs[2] (C3), [3] (C4) and [4] (C5).  One JSON line per
(workload, variant)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from fltee import _lib as L  # noqa: E402
from fltee import device as D  # noqa: E402

for name, steps in (("c3", 200), ("c4", 10), ("c5", 10)):
    for on in (1, 0, 1, 0):
        L.lib().fltee_debug_set_pad_skip(on)
        r = bench.bench_workload(torch, D, name, steps=steps, warmup=3, device=torch.device("cuda", 0))
        print(json.dumps(dict(workload=name, pad_skip=on, kernel_ms=r["kernel_s"] * 1e3,
                              passes=r["net"]["passes"], net_bytes=r["net"]["bytes"])), flush=True)
L.lib().fltee_debug_set_pad_skip(2)

"""A/B in one process: advanced with the fold fused into the compaction's first pass vs
the separate fold pass (fltee_debug_set_fold_compact), at configs[2] (C3) and configs[4]
(C5) shapes.  Prints one JSON line per (shape, variant)."""
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

for name, steps in (("c3", 200), ("c5", 10)):
    w = bench.WORKLOADS[name]
    for fused in (1, 0, 1, 0):
        L.lib().fltee_debug_set_fold_compact(fused)
        r = bench.bench_workload(torch, D, name, steps=steps, warmup=3, device=torch.device("cuda", 0))
        print(json.dumps(dict(workload=name, fused=fused, kernel_ms=r["kernel_s"] * 1e3,
                              passes=r["net"]["passes"], net_bytes=r["net"]["bytes"])), flush=True)
L.lib().fltee_debug_set_fold_compact(1)

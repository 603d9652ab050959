"""A/B of a runtime test hook in ONE process (the same inputs, the same box): the
workload timed by bench.bench_workload with `hook(value)` set before each trial, the
values interleaved, plus the output's bits per value.  One JSON line per (value, repeat).

    python scripts/ab_hook.py c5 fltee_debug_set_swizzle 1 0
(AB_COLD=1: inputs rotated over > 1.5 x the Infinity Cache, as the literal config runs)"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fl-tee_amd")]

import bench  # noqa: E402
from fltee import _lib as L  # noqa: E402
from fltee import device as D  # noqa: E402


def main():
    w, hook, values = sys.argv[1], sys.argv[2], [int(x) for x in sys.argv[3:]]
    reps = int(os.environ.get("AB_REPS", "3"))
    steps = {"c3": 300, "c1": 300, "mnist100": 300}.get(w, 10)
    dev = torch.device("cuda", 0)
    fn = getattr(L.lib(), hook)
    wl = bench.WORKLOADS[w]
    rec = bench.make_records(torch, wl["n"], wl["d"], wl["k"], 1000, dev)
    kw = dict(dense=wl["k"] is None)
    if wl.get("dp"):
        kw.update(seed=7)
    try:
        for rep in range(reps):
            for v in values:
                fn(v)
                r = bench.bench_workload(torch, D, w, steps=steps, warmup=3, device=dev,
                                         cold=os.environ.get("AB_COLD") == "1")
                out = D.aggregate(wl["alg"], rec, wl["n"], wl["k"] or wl["d"], wl["d"], **kw).cpu().numpy()
                h = hashlib.sha256(out.view(np.uint32).tobytes()).hexdigest()[:16]
                print(json.dumps(dict(workload=w, hook=hook, value=v, rep=rep,
                                      kernel_ms=round(r["kernel_s"] * 1e3, 4), out_sha=h,
                                      kernels={k: round(x["ms"] / x["launches"] * 1e3, 1)
                                               for k, x in r["net"]["kernels"].items()})), flush=True)
    finally:
        fn(values[0])


if __name__ == "__main__":
    main()

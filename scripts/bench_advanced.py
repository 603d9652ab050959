"""A/B of the `advanced` second half, interleaved in ONE process.

    python scripts/bench_advanced.py [--workload c5] [--rounds 3] [--launches 3]

Variants: the compaction network with 64 KiB tiles (0) / 32 KiB tiles (1), and the
enclave's second bitonic sort (sort).  Every variant's output is checked bit for bit
against the first; prints one JSON line per variant (median / min ms per aggregate)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from fltee import _lib as L
    from fltee import device as D
    w = bench.WORKLOADS[args.workload]
    n, d, k = w["n"], w["d"], w["k"]
    rec = bench.make_records(torch, n, d, k, 11, "cuda")
    out = torch.empty(d, dtype=torch.float32, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    variants = {"compact64k": (1, 0), "compact32k": (1, 1), "compact32k_64k": (1, 2), "sort": (0, 0)}
    times = {v: [] for v in variants}
    ref = None
    try:
        for _ in range(args.rounds):
            for v, (on, cv) in variants.items():
                L.lib().fltee_debug_set_advanced_compaction(on)
                L.lib().fltee_debug_set_compact_variant(cv)
                D.aggregate(1, rec, n, k, d, out=out, status=st)
                torch.cuda.synchronize()
                o = out.cpu().numpy().view(np.uint32).copy()
                if ref is None:
                    ref = o
                assert np.array_equal(o, ref), f"variant {v} differs"
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.launches):
                    D.aggregate(1, rec, n, k, d, out=out, status=st)
                b.record()
                torch.cuda.synchronize()
                times[v].append(a.elapsed_time(b) / args.launches)
    finally:
        L.lib().fltee_debug_set_advanced_compaction(1)
        L.lib().fltee_debug_set_compact_variant(1)
    assert int(st.item()) == 0
    for v, t in times.items():
        print(json.dumps({"workload": args.workload, "variant": v, "median_ms": float(np.median(t)),
                          "min_ms": float(np.min(t))}), flush=True)


if __name__ == "__main__":
    main()

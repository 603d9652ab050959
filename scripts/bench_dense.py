"""A/B of the dense accumulate variants, interleaved in ONE process (guide §5.4 rule 24).

    python scripts/bench_dense.py [--rounds 7] [--launches 20]
Prints, per variant, the median/min kernel time over rounds and GB/s of algorithmic bytes;
every variant's output is checked bit-for-bit against variant 0."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))
sys.path.insert(0, ROOT)

VARIANTS = {0: "V1 U16 nt 512 lanes (shipped)", 1: "V1 U8 nt", 2: "V1 U32 nt", 3: "V2 U8 nt", 4: "V2 U16 nt",
            5: "V1 U16 plain", 6: "V4 U4 nt", 7: "V4 U8 nt", 8: "= variant 0",
            9: "V1 U16 nt 128 lanes", 10: "8 B/lane U16", 11: "8 B/lane U32", 12: "V1 U16 nt 64 lanes",
            13: "V1 U16 nt 256 lanes (round-1 default)",
            20: "small d: LDS 64 outputs x 32 clients", 21: "small d: LDS 128 x 16",
            22: "small d: LDS 256 x 16", 23: "small d: LDS 64 x 16",
            24: "small d: LDS-DMA ring, 64 outputs x 4 chunks of 16 clients",
            40: "small d: lane per output pair, 100 clients in flight, whole register file",
            41: "small d: the same, 32 in flight", 42: "small d: the same, 64 in flight",
            43: "small d: the same, 50 in flight"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--d", type=int, default=1_000_000)
    ap.add_argument("--buffers", type=int, default=3, help="rotating inputs (10 at MNIST size: cold)")
    ap.add_argument("--variants", default="", help="comma list (default: all)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from fltee import _lib as L
    from fltee import device as D
    n, d = args.n, args.d
    recs = [bench.make_records(torch, n, d, None, 7 + b, "cuda") for b in range(args.buffers)]
    if args.variants:
        keep = {int(v) for v in args.variants.split(",")}
        for v in list(VARIANTS):
            if v not in keep:
                del VARIANTS[v]
    out = torch.empty(d, dtype=torch.float32, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    ref = None
    times = {v: [] for v in VARIANTS}
    for r in range(args.rounds):
        for v in VARIANTS:
            L.lib().fltee_debug_set_dense_variant(v)
            D.aggregate(3, recs[0], n, d, d, out=out, dense=True, status=st)
            torch.cuda.synchronize()
            o = out.cpu().numpy().view(np.uint32).copy()
            if ref is None:
                ref = o
            assert np.array_equal(o, ref), f"variant {v} differs"
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(args.launches):
                D.aggregate(3, recs[i % len(recs)], n, d, d, out=out, dense=True, status=st)
            b.record()
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b) / args.launches)
    L.lib().fltee_debug_set_dense_variant(0)
    assert int(st.item()) == 0
    algo = n * d * 8 + d * 4
    for v, name in VARIANTS.items():
        t = sorted(times[v])
        med = t[len(t) // 2]
        print(json.dumps(dict(variant=v, name=name, median_us=med * 1e3, min_us=t[0] * 1e3,
                              gbs_median=algo / (med / 1e3) / 1e9, frac=algo / (med / 1e3) / 8e12)))


if __name__ == "__main__":
    main()

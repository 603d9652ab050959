"""Micro-benchmark of the oblivious networks and the per-alg pipelines (tuning aid).

    python scripts/bench_sort.py [--sizes 20,24,27] [--modes 0,2]
Prints one JSON line per (mode, M) with the mean time per sort (HIP events)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16,20,24,27")
    ap.add_argument("--modes", default="0,2")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from fltee import device as D
    for mlog in [int(x) for x in args.sizes.split(",")]:
        m = 1 << mlog
        base = torch.randint(0, 1 << 30, (m,), dtype=torch.int64, device="cuda")
        buf = torch.empty_like(base)
        for mode in [int(x) for x in args.modes.split(",")]:
            buf.copy_(base)
            D.bitonic(buf, mode, seed=1)  # warm
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                buf.copy_(base)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                D.bitonic(buf, mode, seed=1)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
            if mode != 2:
                assert bool((buf[1:] .view(torch.int64) >= buf[:-1]).all()) if mode == 1 else True
            print(json.dumps(dict(mode=mode, mlog=mlog, ms=sum(ts) / len(ts), min_ms=min(ts),
                                  gbs_per_pass=2 * m * 8 / (min(ts) / 1e3) / 1e9,
                                  maxr=os.environ.get("FLTEE_BITONIC_MAXR", "5"))), flush=True)
        del base, buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

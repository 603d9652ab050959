"""Position-range sharded `advanced` (Option B) at configs[4] size on ONE GPU with every
range in this process (VirtualRanks: the exchanges are device copies): checks the
result against single-GPU fltee_aggregate_device(advanced) bit for bit and times the
per-range compute.  python scripts/bench_sharded_virtual.py [--worlds 2,4,8]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from fltee import device as D
    from fltee import parallel as P
    n, d, k = 1000, 10_000_000, 100_000
    rec = bench.make_records(torch, n, d, k, 11, "cuda")
    single = D.aggregate(1, rec, n, k, d)
    assert D.status() == 0
    ref = single.cpu().numpy().view(np.uint32).copy()
    nrec = n * k
    M = 1 << (nrec + d - 1).bit_length()
    ops = P.DeviceRangeOps()
    for world, exchange in [(int(x), e) for x in args.worlds.split(",")
                            for e in ("transpose", "pairwise")]:
        C = M // world
        chunks = {r: torch.empty(C, dtype=torch.int64, device="cuda") for r in range(world)}
        comm = P.VirtualRanks(world)
        times = []
        for i in range(args.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for r in range(world):
                D.advanced_init_range(rec[r * C:] if r * C < nrec else rec, nrec, d, r * C, C,
                                      out=chunks[r])
            out = P.index_sharded_advanced(chunks, world, M, n, k, d, ops=ops, comm=comm,
                                           exchange=exchange)
            torch.cuda.synchronize()
            if i:
                times.append(time.perf_counter() - t0)
        same = bool(np.array_equal(out.cpu().numpy().view(np.uint32), ref))
        t = float(np.median(times))
        print(json.dumps(dict(world=world, exchange=exchange, M=M, range_records=C, ms_all_ranks_one_gpu=t * 1e3,
                              ms_per_range_est=t * 1e3 / world, bit_exact_vs_single_gpu=same)),
              flush=True)
        assert same
        del chunks, out


if __name__ == "__main__":
    main()

"""bench_legs.py — the measurement legs bench.py runs.

Every function here times one configuration on the GPU (device-resident unless it says
host-inclusive) or one CPU baseline of the oracle, and returns a dict; bench.py decides
which legs run, writes their full results to a detail file and prints one compact JSON
line (the reference's own harness prints one compact result per run:
secure_aggregation/app/src/benchmark.rs:336-411).
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

WORKLOADS = {
    # name: alg, n clients, d params, k records/client (None = dense, k = d)
    "ns": dict(alg=3, n=100, d=1_000_000, k=None,
               desc="NS: baseline dense fp32 reduce, 100 clients x 1M params"),
    "mnist30": dict(alg=3, n=30, d=50890, k=None,
                    desc="configs[1]: MLP-MNIST num_users=100 frac=0.3 (n=30), baseline, dense"),
    "mnist100": dict(alg=3, n=100, d=50890, k=None,
                     desc="100 clients x MLP-MNIST dense (metric text), baseline"),
    "c1": dict(alg=4, n=30, d=50890, k=5089,
               desc="configs[0] shape on GPU: MLP-MNIST n=30 alpha=0.1, non_oblivious"),
    "c2s": dict(alg=3, n=30, d=50890, k=5089,
                desc="MLP-MNIST n=30 alpha=0.1, baseline on sparse uploads (the ordered sweep)"),
    "b3000": dict(alg=3, n=3000, d=50890, k=5089,
                  desc="the reference's published n=3000 shape, baseline (the ordered sweep)"),
    "a3s": dict(alg=1, n=3, d=50890, k=508,
                desc="exp5's smallest advanced row: MLP-MNIST n=3 alpha=0.01 (M = 2^16)"),
    "a30": dict(alg=1, n=30, d=50890, k=5089,
                desc="exp5's MLP-MNIST n=30 alpha=0.1 advanced row (M = 2^18)"),
    "a300": dict(alg=1, n=300, d=50890, k=508,
                 desc="exp5's MLP-MNIST n=300 alpha=0.01 advanced row (M = 2^18, runs up to 301)"),
    "c3": dict(alg=1, n=100, d=50890, k=5089,
               desc="configs[2]: MLP-MNIST num_users=1000 frac=0.1 alpha=0.1 (n=100), advanced"),
    "c4": dict(alg=2, n=300, d=44964, k=4496, dp=True,
               desc="configs[3]: Purchase100 num_users=1000 frac=0.3 (n=300) alpha=0.1, nips19 + DP"),
    "c5": dict(alg=1, n=1000, d=10_000_000, k=100_000,
               desc="configs[4]: synthetic 10M x 1000 clients (k=1%), advanced"),
}
ALG_NAMES = {1: "advanced", 2: "nips19", 3: "baseline", 4: "non_oblivious", 5: "path_oram", 6: "optimized"}


def make_records(torch, n, d, k, seed, device):
    """Synthetic client records in HBM (int64 = Weight bytes), client-major."""
    g = torch.Generator(device=device).manual_seed(seed)
    if k is None:
        vals = torch.randn(n, d, generator=g, device=device) * 0.01
        idx = torch.arange(d, device=device, dtype=torch.int64).expand(n, d)
    else:
        vals = torch.randn(n, k, generator=g, device=device) * 0.01
        # k distinct indices per client (a run from a random offset, mod d); the
        # oblivious networks' cost does not depend on which indices these are
        j = torch.arange(k, device=device, dtype=torch.int64)
        off = torch.randint(0, d, (n, 1), generator=g, device=device)
        idx = (off + j.unsqueeze(0)) % d
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
    return rec


def time_steps(torch, fn, steps, warmup, stream):
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    # one event pair around the back-to-back launches (per-step pairs would add their own
    # gaps, a large share of a 5-10 us kernel)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record(stream)
    for i in range(steps):
        fn(warmup + i)
    b.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern = a.elapsed_time(b) / steps / 1e3
    return wall, kern


def launch_times(torch, fn, steps, start, stream):
    """per-launch durations (ms): an event pair around each launch, back to back (each
    pair's own gap included — for the distribution, not the headline)"""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(ev):
        a.record(stream)
        fn(start + i)
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def bench_workload(torch, D, name, steps, warmup, device, nbuf=3, cold=False, per_launch=False):
    """cold=True: rotate through enough input buffers (> 1.5 x the 256 MiB Infinity
    Cache) that every launch reads its records from HBM.  per_launch: also each launch's
    own event time (launch_ms)."""
    w = WORKLOADS[name]
    n, d, k = w["n"], w["d"], w["k"]
    kk = d if k is None else k
    bytes_per_step = n * kk * 8
    if cold:
        nbuf = max(nbuf, int(1.5 * 256 * 2 ** 20 // max(bytes_per_step, 1)) + 1)
    nbuf = max(1, min(nbuf, int(2.4e9 // max(bytes_per_step, 1))))  # rotate >=3 when it fits
    recs = [make_records(torch, n, d, k, 1000 + b, device) for b in range(nbuf)]
    out = torch.empty(d, dtype=torch.float32, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    kw = dict(dense=k is None, status=status)
    if w.get("dp"):
        kw.update(dp=True, sigma=1.12, clipping=1.0, seed=7)
    D.reserve(w["alg"], n, kk, d, **{x: y for x, y in kw.items() if x != "status"})
    stream = torch.cuda.current_stream()

    def step(i):
        D.aggregate(w["alg"], recs[i % nbuf], n, kk, d, out=out, **kw)

    wall, kern = time_steps(torch, step, steps, warmup, stream)
    lt = launch_times(torch, step, steps, warmup + steps, stream) if per_launch else None
    assert int(status.item()) == 0, f"device status {int(status.item()):#x}"
    net = net_stats(torch, lambda: step(0))
    del recs
    r = dict(n=n, d=d, k=kk, alg=ALG_NAMES[w["alg"]], wall_s=wall, kernel_s=kern,
             rate=n * kk / kern, bytes=algorithmic_bytes(w), nbuf=nbuf, net=net)
    if lt is not None:
        r["launch_ms"] = lt
    return r


def read_floor(torch, bytes_per_step, device, reps=3, steps=40):
    """The achievable floor beside the metric's literal config: a plain streaming read of
    the same bytes (fltee_debug_read_floor: 16-B non-temporal loads, 8 in flight per lane,
    the grid swept for its best), over buffers rotated past the 256 MiB Infinity Cache
    like the cold literal config's inputs.  Best of `reps` trials per grid, in us."""
    import ctypes as C
    from fltee import _lib as L
    lib = L.lib()
    nbuf = int(1.5 * 256 * 2 ** 20 // max(bytes_per_step, 1)) + 1
    n16 = (bytes_per_step + 15) // 16
    bufs = [torch.empty(n16 * 2, dtype=torch.int64, device=device).random_() for _ in range(nbuf)]
    sink = torch.zeros(8192, dtype=torch.int32, device=device)
    stream = torch.cuda.current_stream()
    best = None
    for blocks in (256, 512, 1024, 2048, 4096):
        def go(i):
            assert lib.fltee_debug_read_floor(C.c_void_p(bufs[i % nbuf].data_ptr()), n16 * 16,
                                              C.c_void_p(sink.data_ptr()), blocks,
                                              C.c_void_p(stream.cuda_stream)) == 0
        for _ in range(reps):
            _, t = time_steps(torch, go, steps, 2 * nbuf, stream)
            if best is None or t < best[0]:
                best = (t, blocks)
    del bufs
    return dict(us=best[0] * 1e6, blocks=best[1], bytes=n16 * 16, gbs=n16 * 16 / best[0] / 1e9,
                input_buffers=nbuf, note="fltee_debug_read_floor: streaming read only, cold "
                                         "(rotated buffers), best grid and trial")


def net_stats(torch, call, reps=3):
    """Streaming passes one aggregate launches and the bytes they sweep (the library's
    launch-side accounting: read + write of the live part of the array per pass, pad-only
    blocks excluded), and per kernel: launches, bytes and time, each launch timed live by
    an event the launcher records on its stream before it (fltee_debug_net_timing; the
    last launch up to a final event).  Best of `reps` aggregates per kernel."""
    from fltee import _lib as L
    lib = L.lib()
    a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
    lib.fltee_debug_net_stats(ctypes.byref(a), ctypes.byref(b), 1)
    call()
    torch.cuda.synchronize()
    lib.fltee_debug_net_stats(ctypes.byref(a), ctypes.byref(b), 1)
    res = dict(passes=a.value, bytes=b.value)
    best = {}
    stream = torch.cuda.current_stream()
    for _ in range(reps):
        torch.cuda.synchronize()
        lib.fltee_debug_net_timing(1, None)
        call()
        lib.fltee_debug_net_timing(0, ctypes.c_void_p(stream.cuda_stream))
        torch.cuda.synchronize()
        per = {}
        name = ctypes.create_string_buffer(64)
        nb, ms = ctypes.c_uint64(0), ctypes.c_float(0)
        n = lib.fltee_debug_net_log(0, None, 0, None, None)
        for i in range(n):
            lib.fltee_debug_net_log(i, name, 64, ctypes.byref(nb), ctypes.byref(ms))
            k = per.setdefault(name.value.decode(), dict(launches=0, bytes=0, ms=0.0))
            k["launches"] += 1
            k["bytes"] += nb.value
            k["ms"] += ms.value
        for k, v in per.items():
            if k not in best or v["ms"] < best[k]["ms"]:
                best[k] = v
    res["kernels"] = best
    return res


def dominant_kernel(net):
    """The kernel with the largest total time in one aggregate (live event timing), its
    bytes per launch (launch-side, pad-aware) and the rate they imply."""
    if not net.get("kernels"):
        return None
    name, k = max(net["kernels"].items(), key=lambda kv: kv[1]["ms"])
    per_launch_ms = k["ms"] / k["launches"]
    bpl = k["bytes"] / k["launches"]
    gbs = bpl / (per_launch_ms * 1e-3) / 1e9
    return dict(kernel=name, launches=k["launches"], bytes_per_launch=bpl, avg_us=per_launch_ms * 1e3,
                achieved_gbs=gbs, frac=gbs / HBM_PEAK_GBS, share_of_aggregate=None)


def rocprof_kernel(name, kernel):
    """Average duration of `kernel` in the newest committed rocprofv3 summary of this
    config (profiles/r0N/<name>_kernel_stats.csv, newest round first), for the
    cross-check, or None."""
    import csv
    paths = [os.path.join(ROOT, "profiles", r, f"{name}_kernel_stats.csv")
             for r in ("r06", "r05", "r04", "r03")]
    path = next((p for p in paths if os.path.exists(p)), paths[-1])
    try:
        with open(path) as f:
            rows = [r for r in csv.DictReader(f) if f"fltee::{kernel}<" in r["Name"] and
                    not (kernel == "bitonic_merge_direct" and ", false, true, " in r["Name"])]
    except (OSError, KeyError):
        return None
    if not rows:
        return None
    calls = sum(int(r["Calls"]) for r in rows)
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    return dict(calls=calls, avg_us=tot / calls / 1e3, source=os.path.relpath(path, ROOT))


def algorithmic_bytes(w):
    """n*k*8 + d*4 (advanced and the flat algorithms), nips19 adds the d*floor(T)
    dummies: (n*k + d*floor(T))*8 + d*4."""
    n, d, k = w["n"], w["d"], w["k"] or w["d"]
    if w["alg"] == 2:
        T = np.float32(2 * k) / np.float32(100.0) * np.float32(np.log(np.float32(d) * np.float32(n)))
        return (n * k + d * int(T)) * 8 + d * 4
    return n * k * 8 + d * 4


def network_records(w):
    """Entries of the array the oblivious network sorts for workload w (0: none)."""
    n, d, k = w["n"], w["d"], w["k"] or w["d"]
    if w["alg"] == 1:
        return 1 << (n * k + d - 1).bit_length()
    if w["alg"] == 2:
        T = np.float32(2 * k) / np.float32(100.0) * np.float32(np.log(np.float32(d) * np.float32(n)))
        return 1 << (n * k + d * int(T) - 1).bit_length()
    return 0


def bench_ns_strong(torch, D, dist, world, rank, device, steps, warmup):
    """The north-star shape FIXED over the node (strong scaling, SURVEY §8e param-range
    shards): 100 clients x 1M dense fp32 params in total, rank r aggregates parameters
    [r*d/N, (r+1)*d/N) of every client (fltee/parallel.py split_dense_columns, rank-local
    indices) and the averaged slices are gathered to rank 0 over RCCL (gather_shards),
    every step.  Timed on every rank (barrier + sync), max over ranks.  Rank 0 also
    aggregates the whole 100 x 1M on its own GPU once, untimed, and compares bit for bit."""
    from fltee import parallel as P
    n, d = 100, 1_000_000
    g = torch.Generator(device=device).manual_seed(4242)  # the same values on every rank
    vals = torch.randn(n, d, generator=g, device=device) * 0.01
    rec, lo, hi = P.split_dense_columns(vals, world, rank)
    dl = hi - lo
    out = torch.empty(dl, dtype=torch.float32, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    D.reserve(3, n, dl, dl, dense=True)
    res = {}

    def step():
        D.aggregate(3, rec, n, dl, dl, out=out, dense=True, status=status)
        return P.gather_shards(out, d, world, rank)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        full = step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert int(status.item()) == 0, f"device status {int(status.item()):#x}"
    if rank == 0:
        one = D.aggregate(3, make_dense_full(torch, vals), n, d, d, dense=True)
        res["bit_identical"] = bool(torch.equal(one.view(torch.int32), full.view(torch.int32)))
        del one
    del rec, vals
    wall = float(t[0]) / steps
    res.update(desc=f"NS 100 x 1M dense baseline FIXED, param-range sharded x{world} + RCCL "
                    "gather of the averaged slices to rank 0 every step",
               alg="baseline", n=n, d=d, ms_per_step=wall * 1e3, value=n * d / wall,
               unit="client-params/s", scaling="strong")
    return res


def make_dense_full(torch, vals):
    """serialize_dense records of values [n][d] (idx = position)."""
    n, d = vals.shape
    idx = torch.arange(d, device=vals.device, dtype=torch.int64).expand(n, d)
    return (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()


def bench_c5_sharded(torch, D, dist, world, rank, device, steps, warmup):
    """configs[4] across the node (SURVEY §8e Option A, strong scaling): C5's 1000
    clients x 100K records over d = 10M are split by client range; every rank runs
    `advanced` on its clients (un-averaged partial), the partials are gathered to rank 0
    over RCCL and summed there in rank order, x 1f32/n (fltee/parallel.py) — the
    reference's alg 6 with batch = n / world.  Timed on every rank, max over ranks."""
    from fltee import parallel as P
    w = WORKLOADS["c5"]
    n, d, k = w["n"], w["d"], w["k"]
    lo, hi = P.shard_range(n, world, rank)
    rec = make_records(torch, hi - lo, d, k, 5000 + rank, device)
    part = torch.empty(d, dtype=torch.float32, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    D.reserve(1, hi - lo, k, d)

    def partial(r, n_, k_, d_):
        return D.aggregate(1, r, n_, k_, d_, out=part, no_average=True, status=status)

    def step():
        P.client_sharded_advanced(rec, hi - lo, k, d, n, world, rank, compute_partial=partial)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert int(status.item()) == 0, f"device status {int(status.item()):#x}"
    del rec
    wall = float(t[0]) / steps
    return dict(desc=w["desc"] + f", client-range sharded x{world} + RCCL gather, rank-order sum",
                alg="advanced", n=n, d=d, k=k, ms_per_step=wall * 1e3, value=n * k / wall,
                unit="client-params/s", scaling="strong")


def bench_c5_index_sharded(torch, D, dist, world, rank, device, steps, warmup,
                           exchange="transpose"):
    """configs[4] as BASELINE.json states it — "param-range sharded across 8 MI355X via
    RCCL/xGMI" (SURVEY §8e Option B, strong scaling): `advanced`'s padded array of
    M = 2^27 entries is split into `world` position ranges; the bitonic network runs
    distributed (range sorts; per stage, two RCCL all-to-alls transpose the rank bits of
    the position into the range so the cross-range steps run locally — or, with
    exchange="pairwise", RCCL exchanges of whole ranges with partner r ^ j/C — then the
    range merges), one halo exchange feeds the
    fold, each rank compacts its run representatives and one RCCL reduce assembles
    the aggregate on rank 0 (fltee/parallel.py).  Rank r holds the records at
    positions [r*C, (r+1)*C) (same synthetic shape as `c5`)."""
    from fltee import parallel as P
    w = WORKLOADS["c5"]
    n, d, k = w["n"], w["d"], w["k"]
    nrec = n * k
    M = 1 << (nrec + d - 1).bit_length()
    C = M // world
    lo = rank * C
    cnt = max(1, min(C, nrec - lo))
    g = torch.Generator(device=device).manual_seed(6000 + rank)
    p = lo + torch.arange(cnt, device=device, dtype=torch.int64)
    off = torch.randint(0, d, (n,), generator=g, device=device)
    idx = (off[torch.clamp(p // k, max=n - 1)] + p % k) % d
    vals = torch.randn(cnt, generator=g, device=device) * 0.01
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).contiguous()
    del p, idx, vals
    chunk = torch.empty(C, dtype=torch.int64, device=device)
    spare = {rank: torch.empty_like(chunk)}
    ops, comm = P.DeviceRangeOps(), P.DistRanks(rank, world)

    def step():
        D.advanced_init_range(rec, nrec, d, lo, C, out=chunk)
        P.index_sharded_advanced({rank: chunk}, world, M, n, k, d, ops=ops, comm=comm,
                                 exchange=exchange, spare=spare)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    del rec, chunk, spare, ops
    wall = float(t[0]) / steps
    how = ("per stage two RCCL all-to-alls transpose the rank bits into the range"
           if exchange == "transpose" else "RCCL pairwise range exchanges")
    return dict(desc=w["desc"] + f", position-range sharded x{world}: distributed bitonic "
                f"({how}) + halo fold + one RCCL reduce", exchange=exchange,
                alg="advanced", n=n, d=d, k=k, M=M, range_records=C, ms_per_step=wall * 1e3,
                value=n * k / wall, unit="client-params/s", scaling="strong")


def bench_c4_index_sharded(torch, D, dist, world, rank, device, steps, warmup):
    """configs[3] (nips19 + DP) by position range ("the same as advanced, the
    shuffle is a bitonic network"; strong scaling): every rank draws the same Laplace
    counts (counter-based Philox, no exchange), builds its range of the padded array,
    the keyed shuffle runs as a distributed network with pairwise RCCL range
    exchanges, each rank selects its entries with idx < d (safe_aggregate's filter, in
    position order), the ragged lists gather on rank 0 in rank order (an all_gather of
    the counts + one gather) and rank 0 adds each index's entries in that order, x
    1f32/n, + DP noise (fltee/parallel.py): bit-identical to one GPU's nips19."""
    from fltee import parallel as P
    w = WORKLOADS["c4"]
    n, d, k, seed = w["n"], w["d"], w["k"], 7
    nrec = n * k
    r, T = D.laplace_r(d, k, n, seed, device=device)
    tf = int(T)
    M = 1 << (nrec + d * tf - 1).bit_length()
    C = M // world
    lo = rank * C
    cnt = max(1, min(C, nrec - lo))
    g = torch.Generator(device=device).manual_seed(7000 + rank)
    p = lo + torch.arange(cnt, device=device, dtype=torch.int64)
    off = torch.randint(0, d, (n,), generator=g, device=device)
    idx = (off[torch.clamp(p // k, max=n - 1)] + p % k) % d
    vals = torch.randn(cnt, generator=g, device=device) * 0.01
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).contiguous()
    del p, idx, vals
    chunk = torch.empty(C, dtype=torch.int64, device=device)
    ops, comm = P.DeviceRangeOps(), P.DistRanks(rank, world)
    dp = dict(sigma=1.12, clipping=1.0, seed=7)

    def step():
        D.laplace_r(d, k, n, seed, device=device)  # each call draws its counts (same seed here)
        D.nips19_build_range(rec, nrec, r, d, tf, lo, C, out=chunk)
        P.index_sharded_nips19({rank: chunk}, world, M, n, d, seed, ops=ops, comm=comm, dp=dp,
                               valid=nrec + d * tf)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    del rec, chunk, ops
    wall = float(t[0]) / steps
    return dict(desc=w["desc"] + f", position-range sharded x{world}: distributed keyed shuffle "
                "(RCCL pairwise range exchanges) + per-range selection + one RCCL gather + in-order sums",
                alg="nips19", n=n, d=d, k=k, M=M, range_records=C, ms_per_step=wall * 1e3,
                value=n * k / wall, unit="client-params/s", scaling="strong")


# The reference's own published bench files for one configuration (SURVEY §6,
# secure_aggregation/results/*-50890-5089-10000-*.txt: d = 50890, k = 5089, 10000 users
# sampled at 0.3 -> n = 3000; "Aggregation" column, seconds, single-threaded SGX enclave).
REF_PUBLISHED = {
    "advanced": dict(alg=1, ref_s=288.2, src="results/advanced-50890-5089-10000-20221121045110UTC.txt"),
    "baseline": dict(alg=3, ref_s=54.3, src="results/baseline-50890-5089-10000-20221121043548UTC.txt"),
    "non_oblivious": dict(alg=4, ref_s=0.456,
                          src="results/non_oblivious-50890-5089-10000-20221121072225UTC.txt"),
    "optimized": dict(alg=6, batch=93, ref_s=10.11, src="results/optimized-93-50890-5089-10000-*.txt (Total)"),
}


def bench_reference_configs(torch, D, device, steps=3):
    """Each algorithm on the exact shape of the reference's published n = 3000 runs,
    device-resident, one GPU; speedup = published enclave seconds / ours."""
    n, d, k = 3000, 50890, 5089
    rec = make_records(torch, n, d, k, 3000, device)
    out = torch.empty(d, dtype=torch.float32, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    res = {}
    for name, r in REF_PUBLISHED.items():
        kw = dict(status=status)
        if "batch" in r:
            kw["batch"] = r["batch"]
        D.aggregate(r["alg"], rec, n, k, d, out=out, **kw)  # warm (grow-only scratch)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(steps):
            D.aggregate(r["alg"], rec, n, k, d, out=out, **kw)
        b.record()
        torch.cuda.synchronize()
        t = a.elapsed_time(b) / steps / 1e3
        res[name] = dict(ms=t * 1e3, ref_s=r["ref_s"], speedup=r["ref_s"] / t, ref_src=r["src"],
                         value=n * k / t, unit="client-params/s")
    assert int(status.item()) == 0, f"device status {int(status.item()):#x}"
    del rec
    return dict(config="d=50890 (MLP-MNIST), k=5089, n=3000 (num_users=10000, ratio 0.3)", **res)


# The reference's headline table: exp/results/exp5.csv column 13 (`execution_time`, the host
# wall time of one Aggregate ECALL, server.rs:140,184-186), driven by exp/exp5.sh:8-48 (frac
# 0.3, --local_skip, --secure_agg); means over the csv's rows per configuration (5 runs, path_oram
# 1-2).  d = the model's parameter count, k = int(alpha * d) (fl_main.py:100-101), n =
# int(0.3 * num_users) sampled clients.
EXP5_MODELS = {"mnist": 50890, "purchase100": 44964}  # MLP (models.py:5-30): 784/600-64-10/100
EXP5_REF_S = {  # (dataset, num_users, alpha) -> {alg: mean execution_time, s}
    ("mnist", 10, 0.1): dict(advanced=0.07196, baseline=0.05707, non_oblivious=0.001405, path_oram=50.35),
    ("mnist", 100, 0.1): dict(advanced=0.1513, baseline=0.5099, non_oblivious=0.003197, path_oram=154.8),
    ("mnist", 1000, 0.1): dict(advanced=2.7725, baseline=5.0185, non_oblivious=0.02831, path_oram=1193.7),
    ("mnist", 10000, 0.1): dict(advanced=287.11, baseline=52.545, non_oblivious=2.5101, path_oram=11962.5),
    ("mnist", 10, 0.01): dict(advanced=0.03041, baseline=0.007275, non_oblivious=0.001159, path_oram=39.56),
    ("mnist", 100, 0.01): dict(advanced=0.06289, baseline=0.05274, non_oblivious=0.001349, path_oram=50.00),
    ("mnist", 1000, 0.01): dict(advanced=0.13796, baseline=0.50328, non_oblivious=0.003354, path_oram=153.9),
    ("mnist", 10000, 0.01): dict(advanced=2.6671, baseline=5.1964, non_oblivious=0.03055, path_oram=1233.7),
    ("purchase100", 100, 0.1): dict(advanced=0.1389, baseline=0.3720, non_oblivious=0.002756, path_oram=139.36),
    ("purchase100", 100, 0.01): dict(advanced=0.03011, baseline=0.03767, non_oblivious=0.001180, path_oram=44.22),
}
EXP5_ALGS = {"advanced": 1, "baseline": 3, "non_oblivious": 4, "path_oram": 5}


def bench_exp5(torch, D, device, reps=5):
    """ecall_secure_aggregation host-inclusive, as exp5 measures it (the host wall time of
    one ECALL: H2D of the ciphertext, GPU AES-CTR, aggregation, D2H of f32[d]), on every
    exp5.csv configuration of the MLP models, beside the reference's published mean.
    Payloads: n clients x k distinct random indices, N(0, 0.01) values, encrypted with the
    clients' session keys (CTR: the library's own kernel), in pageable host memory."""
    from fltee.ecalls import Enclave
    E = Enclave(device.index or 0)
    rows = []
    fl = 9000
    try:
        for (ds, users, alpha), refs in EXP5_REF_S.items():
            d = EXP5_MODELS[ds]
            k = int(alpha * d)
            n = max(int(0.3 * users), 1)
            ids = np.arange(1, n + 1, dtype=np.uint32)
            g = torch.Generator(device=device).manual_seed(users * 7 + k)
            idx = torch.argsort(torch.rand(n, d, generator=g, device=device), dim=1)[:, :k].to(torch.int64)
            vals = torch.randn(n, k, generator=g, device=device) * 0.01
            rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
            cipher = torch.empty_like(rec)
            D.decrypt(ids, rec, k * 8, cipher)  # CTR: encryption == decryption
            host = cipher.cpu().numpy().view(np.uint8)
            del idx, vals, rec, cipher
            for alg, ref_s in refs.items():
                fl += 1
                a = EXP5_ALGS[alg]
                assert E.ecall_fl_init(fl, ids, d, k, 1.12, 1.0, alpha, 1.0, a, 0, 0) == (0, 0)
                walls, phases = [], []
                for r in range(reps + 1):
                    assert E.ecall_start_round(fl, r, n)[:2] == (0, 0)
                    t0 = time.perf_counter()
                    st, rv, out, tt = E.ecall_secure_aggregation(fl, r, ids, host, d, k, a)
                    wall = time.perf_counter() - t0
                    assert (st, rv) == (0, 0), (alg, st, rv)
                    if r:  # the first call grows the staging buffers
                        walls.append(wall)
                        phases.append([float(x) for x in tt])
                t = float(np.mean(walls))
                ph = np.mean(np.array(phases), axis=0) * 1e3
                rows.append(dict(dataset=ds, num_users=users, alpha=alpha, n=n, d=d, k=k, alg=alg,
                                 ms=t * 1e3, min_ms=float(np.min(walls)) * 1e3, ref_ms=ref_s * 1e3,
                                 speedup=ref_s / t, value=n * k / t, unit="client-params/s",
                                 payload_bytes=n * k * 8,
                                 phases_ms=dict(load=float(ph[0]), decrypt=float(ph[1]),
                                                aggregate=float(ph[2]))))
    finally:
        E.destroy()
    return dict(metric="execution_time of one Aggregate ECALL (host wall, server.rs:184-186), "
                       "mean of %d calls after one warm-up" % reps,
                source="reference: exp/results/exp5.csv col 13 means (exp/exp5.sh:8-48)", rows=rows)


def bench_oram_tree(torch, D, device, reps=2):
    """path_oram as the tree Path ORAM (k_oram.hip; oram.rs:64-118: Z = 4, stash 20,
    next_pow2(d) blocks) running the enclave's own access sequence — d prepare writes, a
    read and a write per record in upload order, d readout reads: 2 n k + 2 d accesses —
    on exp5's MLP-MNIST path_oram shapes, device-resident, beside the reference enclave's
    published execution_time for the same configuration (exp5.csv): like for like, access
    for access.  The lazy variant (one read-modify-write per record, blocks created on
    first use, readout by an oblivious sort: n k accesses) is timed beside it."""
    rows = []
    for users, alpha in ((10, 0.1), (100, 0.1), (100, 0.01)):
        d = EXP5_MODELS["mnist"]
        k = int(alpha * d)
        n = max(int(0.3 * users), 1)
        g = torch.Generator(device=device).manual_seed(users + k)
        idx = torch.argsort(torch.rand(n, d, generator=g, device=device), dim=1)[:, :k].to(torch.int64)
        vals = torch.randn(n, k, generator=g, device=device) * 0.01
        rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
        out = torch.empty(d, dtype=torch.float32, device=device)
        ref_s = EXP5_REF_S[("mnist", users, alpha)]["path_oram"]
        row = dict(num_users=users, alpha=alpha, n=n, d=d, k=k, ref_ms=ref_s * 1e3,
                   ref_accesses=2 * n * k + 2 * d)
        for lazy in (False, True):
            D.aggregate(5, rec, n, k, d, out=out, oram_tree=True, oram_lazy=lazy, seed=5)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for r in range(reps):
                D.aggregate(5, rec, n, k, d, out=out, oram_tree=True, oram_lazy=lazy, seed=6 + r)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / reps
            acc = n * k if lazy else 2 * n * k + 2 * d
            if lazy:
                row.update(lazy_accesses=acc, lazy_ms=t * 1e3, lazy_us_per_access=t * 1e6 / acc)
            else:  # the enclave's sequence: the like-for-like speedup
                row.update(accesses=acc, ms=t * 1e3, us_per_access=t * 1e6 / acc, speedup=ref_s / t)
        rows.append(row)
        del rec, idx, vals
    assert D.status() == 0
    return dict(note="tree Path ORAM, one persistent wave (accesses are sequential); `accesses` = "
                     "oram.rs's 2nk + 2d (prepare, read + write per record, readout), the same "
                     "count the enclave's published time covers; lazy: n k accesses + a sorted readout",
                rows=rows)


def bench_next_rows(torch, D, device, steps=5):
    """SURVEY §8f rows on one GPU, device-resident: the GPU AES-128-CTR decrypt of the
    headline payload (lib.rs:312-343) and the client-side producers (utils.py:327-354,
    update.py:187-204, utils.py:268-290) for 100 MLP-MNIST clients at alpha = 0.1."""
    from fltee import client as CL
    res = {}
    n, d = 100, 1_000_000
    ids = np.arange(n, dtype=np.uint32)
    rec = make_records(torch, n, d, None, 41, device)
    cipher = torch.empty_like(rec)
    D.decrypt(ids, rec, d * 8, cipher)  # CTR: encryption == decryption
    plain = torch.empty_like(rec)
    ts = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        D.decrypt(ids, cipher, d * 8, plain)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3)
    assert torch.equal(plain, rec)
    t = min(ts)
    res["aes_ctr_decrypt"] = dict(bytes=n * d * 8, ms=t * 1e3, gbs=2 * n * d * 8 / t / 1e9,
                                  value=n * d / t, unit="client-params/s",
                                  note="100 clients x 8 MB ciphertext -> records (read + write)")
    del rec, cipher, plain
    nc, dc, kc = 100, 50890, 5089
    g = torch.Generator(device=device).manual_seed(43)
    vals = torch.randn(nc, dc, generator=g, device=device) * 0.01
    cids = np.arange(nc, dtype=np.uint32)
    CL.produce_payloads(vals, cids, k=kc, clipping=1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        CL.produce_payloads(vals, cids, k=kc, clipping=1.0)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    res["client_producers"] = dict(ms=t * 1e3, n=nc, d=dc, k=kc, unit="ms per round (all clients)",
                                   note="top-k by |v| + l2clipping + serialize_sparse + AES-CTR, "
                                        "wall time incl. the per-call key upload")
    return res


def cpu_baseline_sample(d, n, seconds):
    """The oracle's `baseline` (baseline.rs o_update: one cmov RMW per 64-B line of the
    d-float output per record) on a bounded prefix of client 0's dense records,
    single thread.  Rate in client-params/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    rng = np.random.default_rng(0)
    m = 256
    spent, done = 0.0, 0
    while spent < seconds:
        w = O.as_weights(np.arange(done, done + m, dtype=np.uint32) % d,
                         rng.normal(0, 0.01, m).astype(np.float32))
        t0 = time.perf_counter()
        O.baseline(w, d, n)
        spent += time.perf_counter() - t0
        done += m
        m = min(m * 2, 1 << 16)
    # context: the enclave's non_oblivious scatter over the FULL workload
    idx = np.tile(np.arange(d, dtype=np.uint32), 1)
    w = O.as_weights(idx, rng.normal(0, 0.01, d).astype(np.float32))
    t0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < 1.0:
        O.non_oblivious(w, d, n)
        reps += 1
    non_obl = reps * d / (time.perf_counter() - t0)
    return dict(value=done / spent, unit="client-params/s", cores=1, kind="port", host=host_cpu(),
                sample=f"oracle baseline (cmov sweep) over {done} records of client 0 into d={d}, "
                       f"{spent:.1f}s, 1 thread",
                non_oblivious_rate=non_obl)


def host_cpu():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return dict(model=model, logical_cpus=os.cpu_count(), cpus_available_to_process=avail)


def _sparse_weights(O, rng, n, d, k):
    idx = np.concatenate([rng.permutation(d)[:k] for _ in range(n)]).astype(np.uint32)
    return O.as_weights(idx, rng.normal(0, 0.01, n * k).astype(np.float32))


def _net_cost(M):
    """compare-exchanges of one bitonic network over M = 2^m entries: M/2 * m(m+1)/2"""
    m = M.bit_length() - 1
    return (M // 2) * m * (m + 1) // 2


def cpu_baseline_configs(gpu_ms):
    """The reference enclave's CPU time per BASELINE.json config, on this host, one
    thread (the enclave has one TCS): the oracle's C restatement of each algorithm
    (advanced at configs[2], nips19 at configs[3], non_oblivious at configs[0],
    baseline at configs[1], advanced at configs[4]), full size where that takes
    seconds, else a bounded sample extrapolated by the oblivious network's
    compare-exchange count (stated per row).  gpu_ms: this run's kernel ms per config."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.set_threads(1)
    rng = np.random.default_rng(1)
    res = {"host": host_cpu(), "threads": 1, "kind": "port"}

    def row(name, n, k, secs, sample, **kw):
        r = dict(n=n, k=k, cpu_s=secs, value=n * k / secs, unit="client-params/s", cores=1,
                 sample=sample, **kw)
        if gpu_ms.get(name):
            r["gpu_ms"] = gpu_ms[name]
            r["gpu_speedup"] = secs * 1e3 / gpu_ms[name]
        res[name] = r

    # configs[0] (C1): non_oblivious, MLP-MNIST n = 30, k = 5089 — full size
    n, d, k = 30, 50890, 5089
    w = _sparse_weights(O, rng, n, d, k)
    t0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < 0.5:
        O.non_oblivious(w, d, n)
        reps += 1
    row("c1", n, k, (time.perf_counter() - t0) / reps, f"full size, mean of {reps} runs")
    # configs[1] (mnist30): baseline (o_update sweep), dense n = 30 x 50890 — sampled prefix
    n, d = 30, 50890
    m = 2048
    wb = O.as_weights(np.arange(m, dtype=np.uint32), rng.normal(0, 0.01, m).astype(np.float32))
    t0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < 2.0:
        O.baseline(wb, d, n)
        reps += 1
    per_rec = (time.perf_counter() - t0) / (reps * m)
    row("mnist30", n, d, per_rec * n * d, f"{reps * m} of the {n * d} records (cost per record "
        "is the same: one cmov per 64-B line of the output), scaled to the full upload")
    # configs[2] (C3): advanced, n = 100, k = 5089, d = 50890 — full size
    n, d, k = 100, 50890, 5089
    w = _sparse_weights(O, rng, n, d, k)
    t0 = time.perf_counter()
    O.advanced(k, w, d, n)
    row("c3", n, k, time.perf_counter() - t0, "full size (two 2^20-entry networks + fold)")
    # configs[3] (C4): nips19, n = 300, k = 4496, d = 44964 — request k / 8 (M = 2^24 instead of
    # 2^27), time scaled by the network's compare-exchange count
    n, d, k = 300, 44964, 4496
    w = _sparse_weights(O, rng, n, d, k)
    ks = k // 8
    Ms = O.next_pow2(n * k + d * int(O.nips19_threshold(d, ks, n)))
    M = O.next_pow2(n * k + d * int(O.nips19_threshold(d, k, n)))
    # the reference's own shuffle: the running FxHash of heap addresses (nips19.rs:66-105,
    # fo_shuffle_fxhash); the keyed comparator the GPU and the oracle share is timed beside it
    t0 = time.perf_counter()
    O.nips19(ks, w, d, n, seed=7, reference_shuffle=True)
    ts = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.nips19(ks, w, d, n, seed=7)
    tk = time.perf_counter() - t0
    scale = _net_cost(M) / _net_cost(Ms)
    row("c4", n, k, ts * scale,
        f"nips19 (the reference's FxHash-of-addresses shuffle network) with request k = {ks} "
        f"(M = {Ms} instead of {M}): {ts:.2f} s measured, x{scale:.2f} (compare-exchange ratio)",
        measured_s=ts, M=M, keyed_shuffle_cpu_s=tk * scale, keyed_shuffle_measured_s=tk)
    # configs[4] (C5): advanced, 1000 x 100K over d = 10M (M = 2^27) — 1/16 of d and k
    n, d, k = 1000, 10_000_000, 100_000
    ns_, ds, ks = 1000, d // 16, k // 16
    idx = (rng.integers(0, ds, ns_)[:, None] + np.arange(ks)[None, :]) % ds
    w = O.as_weights(idx.reshape(-1).astype(np.uint32), rng.normal(0, 0.01, ns_ * ks).astype(np.float32))
    Ms, M = O.next_pow2(ns_ * ks + ds), O.next_pow2(n * k + d)
    t0 = time.perf_counter()
    O.advanced(ks, w, ds, ns_)
    ts = time.perf_counter() - t0
    row("c5", n, k, ts * _net_cost(M) / _net_cost(Ms),
        f"advanced at 1/16 scale (d = {ds}, k = {ks}, M = {Ms}): {ts:.2f} s measured, "
        f"x{_net_cost(M) / _net_cost(Ms):.2f} (compare-exchange ratio of the two networks)",
        measured_s=ts, M=M)
    return res


def e2e_sample(torch, D, n, d, device, reps=3):
    """Host-inclusive rate of the drop-in path: ecall_secure_aggregation with the
    ciphertext in (pageable) host memory, as the Rust host hands it over:
    H2D + GPU AES-CTR decrypt + aggregate + D2H of f32[d].  The ciphertext is made
    with the library's own CTR kernel (CTR encryption == decryption)."""
    from fltee.ecalls import Enclave
    ids = np.arange(n, dtype=np.uint32)
    rec = make_records(torch, n, d, None, 99, device)
    cipher = torch.empty_like(rec)
    D.decrypt(ids, rec, d * 8, cipher)
    host = cipher.cpu().numpy().view(np.uint8)
    expect = D.aggregate(3, rec, n, d, d, dense=True).cpu().numpy()
    del rec, cipher
    E = Enclave(device.index or 0)
    st, rv = E.ecall_fl_init(0, ids, d, d, 1.12, 1.0, 0.1, 1.0, 3, 0, 0)
    assert (st, rv) == (0, 0)
    E.ecall_start_round(0, 0, n)
    walls, phases = [], []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        st, rv, out, tt = E.ecall_secure_aggregation(0, r, ids, host, d, d, 3)
        wall = time.perf_counter() - t0
        assert (st, rv) == (0, 0) and np.array_equal(out.view(np.uint32), expect.view(np.uint32))
        E.ecall_start_round(0, r + 1, n)
        if r:  # first call warms the staging buffers, like benchmark.rs:355-359
            walls.append(wall)
            phases.append(tt.tolist())
    E.destroy()
    wall = float(np.mean(walls))
    ph = np.mean(np.array(phases), axis=0)
    return dict(value=n * d / wall, unit="client-params/s", ms_per_call=wall * 1e3,
                load_ms=ph[0] * 1e3, decrypt_ms=ph[1] * 1e3, aggregate_ms=ph[2] * 1e3,
                bytes_h2d=n * d * 8, note="ecall_secure_aggregation, pageable host ciphertext, "
                "times = execution_time_results {load = H2D (AES pipelined under it), decrypt = "
                "AES left after the last chunk landed, aggregate+D2H}")


def c_abi_multi_gpu(world, timeout=420):
    """The multi-GPU path as the Rust host reaches it: ECALLs on one enclave id over all
    `world` GPUs (fltee_device_init_multi), host-inclusive, vs a one-GPU eid
    (scripts/ecall_multi_bench.py).  Run in a child process: it opens its own RCCL
    communicators over the node's GPUs while this job's ranks wait on a host barrier."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "ecall_multi_bench.py"), "--devices",
           str(world)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    except Exception as ex:  # noqa: BLE001 - reported, never fatal for the bench line
        return {"error": repr(ex)}
    lines = [x for x in r.stdout.strip().splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc={r.returncode}", "stderr": r.stderr[-1500:]}
    return json.loads(lines[-1])


def _build_id():
    """fltee_version(): the source hash the loaded library was built from (provenance)."""
    from fltee import _lib as L
    return L.lib().fltee_version().decode()


def traffic_from_profiles(name):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        return t[name]["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None



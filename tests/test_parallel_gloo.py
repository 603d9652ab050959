"""N>1 path on CPU: two gloo ranks run fltee.parallel's sharding + collectives with
the oracle standing in for the HIP kernels, and must reproduce the single-process
oracle result bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def data():
    rng = np.random.default_rng(42)
    n, d = 5, 101
    dense = rng.normal(0, 0.01, (n, d)).astype(np.float32)
    nc, dk, k = 6, 300, 20
    idx = np.concatenate([rng.choice(dk, k, replace=False) for _ in range(nc)]).astype(np.uint32)
    val = rng.normal(0, 0.01, nc * k).astype(np.float32)
    return dense, (nc, dk, k, idx, val)


def worker(rank, world, port, outdir):
    import sys
    for p in (ROOT, os.path.join(ROOT, "fl-tee_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    from fltee import parallel as P
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    dense, (nc, dk, k, idx, val) = data()
    n, d = dense.shape

    # ---- parameter-range sharding (dense baseline) ----
    rec, lo, hi = P.split_dense_columns(torch.from_numpy(dense), world, rank)

    def compute(records, n_, d_):
        r = records.numpy().view(np.uint64)
        w = O.as_weights((r & 0xFFFFFFFF).astype(np.uint32),
                         (r >> 32).astype(np.uint32).view(np.float32))
        return torch.from_numpy(O.baseline(w, d_, n_))

    full = P.param_sharded_dense(rec, n, hi - lo, d, world, rank, compute=compute)

    # ---- client-range sharding (advanced, Option A) ----
    c0, c1 = P.shard_range(nc, world, rank)

    def compute_partial(records, n_, k_, d_):
        s, st = O.advanced_core(k_, d_, records, n_)
        assert st == 0
        return torch.from_numpy(s["val"][:d_].copy())

    def combine(rows, coef):
        acc = np.zeros(rows.shape[1], np.float32)
        for r in rows.numpy():          # rank order == alg-6 batch order
            acc = acc + r
        return torch.from_numpy(acc * np.float32(coef))

    local = O.as_weights(idx[c0 * k:c1 * k], val[c0 * k:c1 * k])
    adv = P.client_sharded_advanced(local, c1 - c0, k, dk, nc, world, rank,
                                    compute_partial=compute_partial, combine=combine)
    if rank == 0:
        np.save(os.path.join(outdir, "dense.npy"), full.numpy())
        np.save(os.path.join(outdir, "adv.npy"), adv.numpy())
    else:
        assert full is None and adv is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_paths_match_single_process(oracle, tmp_path, world):
    mp.spawn(worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    dense, (nc, dk, k, idx, val) = data()
    n, d = dense.shape
    w = oracle.as_weights(np.tile(np.arange(d, dtype=np.uint32), n), dense.reshape(-1))
    ref_dense = oracle.baseline(w, d, n)
    got = np.load(tmp_path / "dense.npy")
    assert np.array_equal(got.view(np.uint32), ref_dense.view(np.uint32))
    # equal client shards == alg 6 with batch = n / world (lib.rs:498-573), bit for bit
    if nc % world == 0:
        ref_adv, st = oracle.client_size_optimized(nc // world, k, oracle.as_weights(idx, val), dk, nc)
        assert st == 0
        got = np.load(tmp_path / "adv.npy")
        assert np.array_equal(got.view(np.uint32), ref_adv.view(np.uint32))


def test_shard_ranges_cover():
    from fltee.parallel import shard_range
    for total in (1, 7, 100, 1_000_003):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


# ---- position-range sharding (advanced, Option B): DistRanks over gloo ----
def case_b():
    rng = np.random.default_rng(7)
    n, d, k = 6, 300, 40
    idx = np.concatenate([rng.choice(d, k, replace=False) for _ in range(n)]).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    return n, d, k, idx, val


def worker_b(rank, world, port, outdir, exchange):
    import sys
    for p in (ROOT, os.path.join(ROOT, "fl-tee_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    from range_ops_np import NumpyRangeOps, init_range

    from fltee import parallel as P
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    n, d, k, idx, val = case_b()
    M = 1 << (n * k + d - 1).bit_length()
    C = M // world
    chunks = {rank: init_range(idx, val, d, rank * C, C)}
    out = P.index_sharded_advanced(chunks, world, M, n, k, d, ops=NumpyRangeOps(),
                                   comm=P.DistRanks(rank, world), exchange=exchange)
    if rank == 0:
        np.save(os.path.join(outdir, "adv_b.npy"), out.numpy())
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["transpose", "pairwise"])
@pytest.mark.parametrize("world", [2, 4])
def test_index_sharded_advanced_gloo(oracle, tmp_path, world, exchange):
    mp.spawn(worker_b, args=(world, free_port(), str(tmp_path), exchange), nprocs=world, join=True)
    n, d, k, idx, val = case_b()
    ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
    assert st == 0
    got = np.load(tmp_path / "adv_b.npy")
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


# ---- position-range sharded nips19: DistRanks.gather_lists over gloo ----
NIPS_SEED = 0x1234_0000_00C0_FFEE


def case_c():
    rng = np.random.default_rng(11)
    m, d, n = 1024, 50, 7
    idx = rng.integers(0, 80, m).astype(np.uint32)  # idx >= d: pads/dummies, dropped
    val = rng.normal(0, 0.01, m).astype(np.float32)
    return m, d, n, idx, val


def worker_c(rank, world, port, outdir):
    import sys
    for p in (ROOT, os.path.join(ROOT, "fl-tee_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import oracle as O
    from range_ops_np import NumpyRangeOps

    from fltee import parallel as P
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    m, d, n, idx, val = case_c()
    full = torch.from_numpy(O.as_weights(idx, val).view(np.int64).copy())
    C = m // world
    chunks = {rank: full[rank * C:(rank + 1) * C].clone()}
    out = P.index_sharded_nips19(chunks, world, m, n, d, NIPS_SEED, ops=NumpyRangeOps(),
                                 comm=P.DistRanks(rank, world))
    if rank == 0:
        np.save(os.path.join(outdir, "nips.npy"), out.numpy())
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_index_sharded_nips19_gloo(oracle, tmp_path, world):
    """Ragged per-rank selections gathered in rank order == the single-array keyed
    shuffle + in-order safe_aggregate (nips19.rs:51-61, common.rs:25-35), bit for bit."""
    mp.spawn(worker_c, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    m, d, n, idx, val = case_c()
    key = (NIPS_SEED ^ (NIPS_SEED >> 32)) & 0xFFFFFFFF
    s = oracle.shuffle_keyed(oracle.as_weights(idx, val), key)
    ref = oracle.safe_aggregate(s, d, n)
    got = np.load(tmp_path / "nips.npy")
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))

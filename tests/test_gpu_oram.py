"""path_oram as a tree Path ORAM on the GPU (k_oram.hip; oram.rs:64-118: Z = 4, stash 20,
next_pow2(d) blocks, one read + write per uploaded record in upload order, then d reads).

The ORAM's placement is random (per-call seed), its output is not: the in-order f32 sum
of each index's values from +0.0, x 1f32/n — bit for bit the oracle's fo_path_oram (and
so non_oblivious / baseline / the sweep).  Parity unpinned against the crate itself
(mc-oblivious-ram is not vendored in the reference): pinned to its call sites' semantics.
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


@pytest.fixture(scope="module")
def dev():
    import torch

    from fltee import device as D
    torch.cuda.init()
    return D


def cuda_records(D, idx, val):
    import torch
    return torch.from_numpy(D.pack_records(idx, val)).cuda()


def bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("n,d,k,dup", [(1, 1, 1, False), (2, 2, 2, True), (3, 17, 9, False),
                                       (4, 1000, 300, True), (7, 4099, 700, False),
                                       (30, 50890, 5089, False), (5, 65536, 3000, True)])
def test_tree_oram_bit_exact(dev, oracle, n, d, k, dup):
    """Sparse uploads (dup: indices repeated inside a client, and every index of
    [d, next_pow2(d)) the ORAM holds but never reads back) == fo_path_oram, bit for bit;
    two seeds (different trees) give the same bits."""
    rng = np.random.default_rng(n * 7 + d)
    cap = 1 << (d - 1).bit_length() if d > 1 else 1
    if dup:
        idx = rng.integers(0, cap, n * k).astype(np.uint32)
    else:
        idx = np.concatenate([rng.permutation(d)[:k] for _ in range(n)]).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    val[::97] = -0.0  # +0.0 + -0.0 = +0.0: the enclave's first add
    rec = cuda_records(dev, idx, val)
    ref, st = oracle.path_oram(oracle.as_weights(idx, val), d, n)
    assert st == 0
    for seed in (11, 12):
        out = dev.aggregate(5, rec, n, k, d, oram_tree=True, seed=seed).cpu().numpy()
        assert dev.status() == 0
        assert bits_equal(out, ref)


def test_tree_oram_dense_and_accumulate(dev, oracle):
    """Dense uploads run through the ORAM too (n*d accesses); accumulate adds the sums."""
    import torch
    n, d = 3, 3000
    rng = np.random.default_rng(3)
    idx = np.tile(np.arange(d, dtype=np.uint32), n)
    val = rng.normal(0, 0.01, n * d).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    ref, st = oracle.path_oram(oracle.as_weights(idx, val), d, n)
    out = dev.aggregate(5, rec, n, d, d, dense=True, oram_tree=True).cpu().numpy()
    assert dev.status() == 0 and bits_equal(out, ref)
    base = torch.full((d,), 0.25, dtype=torch.float32, device="cuda")
    dev.aggregate(5, rec, n, d, d, out=base, accumulate=True, oram_tree=True)
    sums, _ = oracle.path_oram(oracle.as_weights(idx, val), d, 1)
    assert bits_equal(base.cpu().numpy(), np.float32(0.25) + sums)


def test_tree_oram_out_of_range_and_too_large(dev):
    """idx >= next_pow2(d) is an ORAM access out of range (the crate panics): the index
    range bit; next_pow2(d) > 2^16 blocks (the LDS position map) is refused."""
    rec = cuda_records(dev, np.array([0, 1024], np.uint32), np.array([1, 1], np.float32))
    dev.aggregate(5, rec, 1, 2, 1000, oram_tree=True)
    assert dev.status() & 0x2
    rec = cuda_records(dev, np.array([0], np.uint32), np.array([1], np.float32))
    with pytest.raises(RuntimeError):
        dev.aggregate(5, rec, 1, 1, 65537, oram_tree=True)


def test_tree_oram_through_the_ecall(oracle):
    """fltee_set_path_oram_tree(1): the ECALL's alg 5 runs the tree ORAM, and returns the
    same bits as the sweep (the default) and as the oracle enclave."""
    import torch

    from fltee.ecalls import Enclave, set_path_oram_tree
    torch.cuda.init()
    n, d, k = 6, 2000, 400
    rng = np.random.default_rng(9)
    ids = np.arange(30, 30 + n, dtype=np.uint32)
    recs = []
    for _ in range(n):
        w = np.zeros(k, dtype=oracle.WEIGHT)
        w["idx"] = rng.permutation(d)[:k]
        w["val"] = rng.normal(0, 0.01, k).astype(np.float32)
        recs.append(w)
    enc = oracle.encrypt_clients(ids, [r.tobytes() for r in recs])
    E = Enclave(0)
    outs = []
    try:
        for fl, tree in ((880, False), (881, True)):
            set_path_oram_tree(tree)
            assert E.ecall_fl_init(fl, ids, d, k, 1.12, 1.0, 0.1, 1.0, 5, 0, 0) == (0, 0)
            assert E.ecall_start_round(fl, 0, n)[:2] == (0, 0)
            st, rv, out, _ = E.ecall_secure_aggregation(fl, 0, ids, enc, d, k, 5)
            assert (st, rv) == (0, 0)
            outs.append(out)
    finally:
        set_path_oram_tree(False)
        E.destroy()
    ref, st = oracle.path_oram(oracle.as_weights(np.concatenate([r["idx"] for r in recs]),
                                                 np.concatenate([r["val"] for r in recs])), d, n)
    assert st == 0 and bits_equal(outs[0], ref) and bits_equal(outs[1], ref)

"""path_oram as a tree Path ORAM on the GPU (k_oram.hip; oram.rs:64-118: Z = 4, stash 20,
next_pow2(d) blocks; by default oram.rs's own access sequence — d prepare writes, a read and
a write per uploaded record in upload order, then d reads — and with oram_lazy one
read-modify-write per record and the oblivious readout).

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


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("n,d,k,dup", [(1, 1, 1, False), (2, 2, 2, True), (3, 17, 9, False),
                                       (4, 1000, 300, True), (7, 4099, 700, False),
                                       (30, 50890, 5089, False), (5, 65536, 3000, True),
                                       (3, 131072, 500, True)])
def test_tree_oram_bit_exact(dev, oracle, n, d, k, dup, lazy):
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
        out = dev.aggregate(5, rec, n, k, d, oram_tree=True, oram_lazy=lazy, seed=seed).cpu().numpy()
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
    for lazy in (False, True):
        out = dev.aggregate(5, rec, n, d, d, dense=True, oram_tree=True, oram_lazy=lazy).cpu().numpy()
        assert dev.status() == 0 and bits_equal(out, ref)
        base = torch.full((d,), 0.25, dtype=torch.float32, device="cuda")
        dev.aggregate(5, rec, n, d, d, out=base, accumulate=True, oram_tree=True, oram_lazy=lazy)
        sums, _ = oracle.path_oram(oracle.as_weights(idx, val), d, 1)
        assert bits_equal(base.cpu().numpy(), np.float32(0.25) + sums)


def test_tree_oram_out_of_range_and_too_large(dev):
    """idx >= next_pow2(d) is an ORAM access out of range (the crate panics): the index
    range bit; next_pow2(d) > 2^22 blocks (the path no longer fits one wave) is refused by
    the device call (the ECALL takes the sweep there: test_tree_oram_ecall_large_d)."""
    rec = cuda_records(dev, np.array([0, 1024], np.uint32), np.array([1, 1], np.float32))
    dev.aggregate(5, rec, 1, 2, 1000, oram_tree=True)
    assert dev.status() & 0x2
    rec = cuda_records(dev, np.array([0], np.uint32), np.array([1], np.float32))
    with pytest.raises(RuntimeError):
        dev.aggregate(5, rec, 1, 1, (1 << 22) + 1, oram_tree=True)


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


def test_tree_oram_one_million_blocks(dev, oracle):
    """d = 1M (N = 2^20 blocks, 21-level paths): no LDS position map any more — the leaves
    come from the oblivious precompute.  oram.rs's sequence (2 n k + 2 d = 2,000,600
    accesses) and the lazy one, bit for bit the in-order sum."""
    n, d, k = 2, 1_000_000, 150
    rng = np.random.default_rng(77)
    idx = rng.integers(0, d, n * k).astype(np.uint32)
    idx[5] = idx[3]  # a repeat inside client 0
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    ref, st = oracle.path_oram(oracle.as_weights(idx, val), d, n)
    assert st == 0
    for lazy in (True, False):
        out = dev.aggregate(5, rec, n, k, d, oram_tree=True, oram_lazy=lazy, seed=3).cpu().numpy()
        assert dev.status() == 0
        assert bits_equal(out, ref)


@pytest.mark.parametrize("dense", [False, True])
def test_tree_oram_clip_equals_sweep(dev, dense):
    """The server-side clip (update.py:187-204) applies to the records the tree reads,
    dense or sparse: the same bits as the clipped sweep / dense kernel."""
    n, d = 5, 700
    k = d if dense else 90
    rng = np.random.default_rng(8 + dense)
    if dense:
        idx = np.tile(np.arange(d, dtype=np.uint32), n)
    else:
        idx = np.concatenate([rng.permutation(d)[:k] for _ in range(n)]).astype(np.uint32)
    val = rng.normal(0, 0.5, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    want = dev.aggregate(5, rec, n, k, d, dense=dense, clip=True, clipping=0.3).cpu().numpy()
    assert dev.status() == 0
    for lazy in (False, True):
        got = dev.aggregate(5, rec, n, k, d, dense=dense, clip=True, clipping=0.3, oram_tree=True,
                            oram_lazy=lazy).cpu().numpy()
        assert dev.status() == 0
        assert bits_equal(got, want)
    plain = dev.aggregate(5, rec, n, k, d, dense=dense, oram_tree=True).cpu().numpy()
    assert not bits_equal(plain, want)  # the clip did something


def test_tree_oram_stash_overflow_reported(dev, oracle):
    """fltee_debug_set_oram_bucket(0): no bucket takes a block, so every block stays in the
    20-entry stash and the 21st distinct block overflows it: the device status bit, and
    the ECALL's 0x1 (SGX_ERROR_UNEXPECTED; the crate panics)."""
    from fltee import _lib as L
    from fltee.ecalls import Enclave, set_path_oram_tree
    rng = np.random.default_rng(1)
    n, d, k = 1, 64, 30
    idx = rng.permutation(d)[:k].astype(np.uint32)
    val = rng.normal(0, 1, k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    ids = np.array([7], np.uint32)
    w = oracle.as_weights(idx, val)
    enc = oracle.encrypt_clients(ids, [w.tobytes()])
    E = Enclave(0)
    try:
        L.lib().fltee_debug_set_oram_bucket(0)
        dev.aggregate(5, rec, n, k, d, oram_tree=True)
        assert dev.status() & 0x8
        set_path_oram_tree(True)
        assert E.ecall_fl_init(870, ids, d, k, 1.12, 1.0, 0.1, 1.0, 5, 0, 0) == (0, 0)
        assert E.ecall_start_round(870, 0, n)[:2] == (0, 0)
        st, rv, out, _ = E.ecall_secure_aggregation(870, 0, ids, enc, d, k, 5)
        assert (st, rv) == (0, L.ERROR_UNEXPECTED) and not out.any()
    finally:
        L.lib().fltee_debug_set_oram_bucket(4)
        set_path_oram_tree(False)
        E.destroy()
    out = dev.aggregate(5, rec, n, k, d, oram_tree=True).cpu().numpy()  # the knob restored
    assert dev.status() == 0
    ref, _ = oracle.path_oram(w, d, n)
    assert bits_equal(out, ref)


def test_tree_oram_ecall_multi_gpu_eid_and_large_d(oracle):
    """The tree through the ECALL on a multi-GPU eid (dense uploads: the root runs the
    tree instead of the group's dense shards) == the single-GPU eid == the oracle; and a
    d past the tree's 2^22 blocks takes the sweep (plan and behaviour agree)."""
    import torch

    from fltee.ecalls import Enclave, set_path_oram_tree
    torch.cuda.init()
    n, d = 4, 900
    rng = np.random.default_rng(2)
    ids = np.arange(40, 40 + n, dtype=np.uint32)
    plain = []
    for _ in ids:
        w = np.zeros(d, dtype=oracle.WEIGHT)
        w["idx"] = np.arange(d)
        w["val"] = rng.normal(0, 0.01, d).astype(np.float32)
        plain.append(w)
    enc = oracle.encrypt_clients(ids, [p.tobytes() for p in plain])
    ref, _ = oracle.path_oram(np.concatenate(plain), d, n)
    outs = []
    set_path_oram_tree(True)
    try:
        for devs in (0, [0, 0]):
            E = Enclave(devs)
            try:
                fl = 850 + len(outs)
                assert E.ecall_fl_init(fl, ids, d, d, 1.12, 1.0, 0.1, 1.0, 5, 0, 0) == (0, 0)
                assert E.ecall_start_round(fl, 0, n)[:2] == (0, 0)
                st, rv, out, _ = E.ecall_secure_aggregation(fl, 0, ids, enc, d, d, 5)
                assert (st, rv) == (0, 0)
                outs.append(out)
                if devs == 0:  # d beyond the tree: the sweep
                    big = (1 << 22) + 3
                    one = oracle.as_weights(np.array([big - 1], np.uint32), np.array([2.5], np.float32))
                    enc1 = oracle.encrypt_clients(ids[:1], [one.tobytes()])
                    assert E.ecall_fl_init(860, ids[:1], big, 1, 1.12, 1.0, 0.1, 1.0, 5, 0, 0) == (0, 0)
                    assert E.ecall_start_round(860, 0, 1)[:2] == (0, 0)
                    st, rv, ob, _ = E.ecall_secure_aggregation(860, 0, ids[:1], enc1, big, 1, 5)
                    assert (st, rv) == (0, 0) and ob[big - 1] == 2.5 and np.count_nonzero(ob) == 1
            finally:
                E.destroy()
    finally:
        set_path_oram_tree(False)
    assert bits_equal(outs[0], ref) and bits_equal(outs[1], ref)

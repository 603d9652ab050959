"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-exact for indices / permutations and for every aggregation whose
reference order we reproduce (dense + sparse flat algorithms, advanced, alg 6);
nips19 (Laplace counts, keyed shuffle, in-order safe_aggregate) is bit-exact too;
the DP noise is checked statistically and against the oracle's draws.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

U32MAX = 0xFFFFFFFF


@pytest.fixture(scope="module")
def dev():
    import torch

    from fltee import device as D
    torch.cuda.init()
    return D


def cuda_records(D, idx, val):
    import torch
    return torch.from_numpy(D.pack_records(idx, val)).cuda()


def rand_sparse(rng, n, d, k, scale=0.01):
    idx = np.concatenate([rng.choice(d, k, replace=False) for _ in range(n)]).astype(np.uint32)
    val = rng.normal(0, scale, n * k).astype(np.float32)
    return idx, val


def bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


# ------------------------------------------------------- flat algorithms ----
@pytest.mark.parametrize("n,d", [(1, 2), (3, 7), (5, 1000), (30, 50890), (2, 65537), (17, 4099),
                                 (100, 50890), (70, 50891), (33, 300000), (64, 50890), (99, 1000),
                                 (40, 2002)])
@pytest.mark.parametrize("alg", [3, 4, 5])
def test_dense_bit_exact(dev, oracle, n, d, alg):
    rng = np.random.default_rng(n * 1000 + d)
    idx = np.tile(np.arange(d, dtype=np.uint32), n)
    val = rng.normal(0, 0.01, n * d).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(alg, rec, n, d, d, dense=True).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.non_oblivious(oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)


@pytest.mark.parametrize("n,d", [(100, 50890), (45, 1001), (3, 130), (16, 2048), (65, 4096),
                                 (1000, 256), (30, 50890)])
@pytest.mark.parametrize("clip,acc", [(True, False), (False, True), (True, True)])
def test_dense_small_d_kernel_equals_streaming_kernel(dev, n, d, clip, acc):
    """The small-d kernels (variant 0's default: the whole-batch kernel for 32 < n <= 100,
    else register-staged LDS chunks; the LDS-DMA ring, variant 24; the whole-batch kernel
    with clamped batches of 100 / 32, variants 40 / 41) == the one-lane-per-pair streaming
    kernel (variant 13), bit for bit, with the per-client clip and accumulate fused;
    partial and whole chunks of 16 / 32 clients, a partial last block of outputs."""
    import torch

    from fltee import _lib as L
    rng = np.random.default_rng(n + d)
    idx = np.tile(np.arange(d, dtype=np.uint32), n)
    val = rng.normal(0, 0.01, n * d).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    prev = torch.from_numpy(rng.normal(0, 1, d).astype(np.float32)).cuda()
    outs = []
    try:
        for variant in (0, 13, 24, 40, 41):
            L.lib().fltee_debug_set_dense_variant(variant)
            out = prev.clone()
            dev.aggregate(3, rec, n, d, d, out=out, dense=True, clip=clip, clipping=0.5,
                          accumulate=acc)
            assert dev.status() == 0
            outs.append(out.cpu().numpy())
    finally:
        L.lib().fltee_debug_set_dense_variant(0)
    assert all(bits_equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("n,d", [(2, 64), (50, 2000), (100, 50890)])
def test_dense_order_violation_is_reported(dev, n, d):
    idx = np.tile(np.arange(d, dtype=np.uint32), n)
    idx[d + 6] = 3
    rec = cuda_records(dev, idx, np.ones(n * d, np.float32))
    dev.aggregate(3, rec, n, d, d, dense=True)
    assert dev.status() & 0x1


# (2, 2M, 100): non_oblivious takes the stable-sort path (the [n][d] scatter rows would
# cost more than the sort); the others take the scatter-rows path
@pytest.mark.parametrize("n,d,k", [(1, 10, 3), (4, 1000, 100), (30, 50890, 5089), (7, 3001, 2999),
                                   (2, 2_000_000, 100)])
@pytest.mark.parametrize("alg", [3, 4, 5])
def test_sparse_bit_exact(dev, oracle, n, d, k, alg):
    rng = np.random.default_rng(n + d + k)
    idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(alg, rec, n, k, d).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.non_oblivious(oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)


@pytest.mark.parametrize("alg", [3, 4, 5])
def test_sparse_repeated_index_exact(dev, alg):
    # baseline / path_oram's ordered sweep and non_oblivious's scatter: exact, no flag
    idx = np.array([1, 1, 2, 3], np.uint32)
    rec = cuda_records(dev, idx, np.ones(4, np.float32))
    out = dev.aggregate(alg, rec, 2, 2, 8).cpu().numpy()
    assert dev.status() == 0
    assert out.tolist() == [0, 1.0, 0.5, 0.5, 0, 0, 0, 0]


@pytest.mark.parametrize("n,d,k", [(3, 700, 300), (30, 50890, 5089), (5, 70000, 3000), (2, 1_100_000, 200)])
@pytest.mark.parametrize("alg", [3, 5])
def test_sweep_ordered_repeats_bit_exact(dev, oracle, n, d, k, alg):
    """The ordered sweep (baseline / path_oram on sparse uploads) against the oracle's
    in-order sum with heavy repeats inside clients (runs of up to k of one index), the
    64-lane and 256-lane block shapes, partial chunks, accumulate."""
    import torch
    rng = np.random.default_rng(n * 7 + k)
    idx = rng.integers(0, min(d, 97), n * k).astype(np.uint32)  # many repeats
    idx[::3] = rng.integers(0, d, len(idx[::3])).astype(np.uint32)
    val = rng.normal(0, 1, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(alg, rec, n, k, d).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.non_oblivious(oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)
    prev = torch.from_numpy(rng.normal(0, 1, d).astype(np.float32)).cuda()
    acc = prev.clone()
    dev.aggregate(alg, rec, n, k, d, out=acc, accumulate=True)
    assert dev.status() == 0
    sums, _ = oracle.non_oblivious(oracle.as_weights(idx, val), d, 1)
    assert bits_equal(acc.cpu().numpy(), prev.cpu().numpy() + sums)


def test_non_oblivious_scatter_repeat_flag_is_per_call(dev, oracle):
    """The scatter's repeated-index mark is tagged with the call's epoch: a call with a
    repeated index, then calls without, then with again, each exact (no stale flag)."""
    rng = np.random.default_rng(3)
    n, d, k = 6, 700, 90
    good_i, good_v = rand_sparse(rng, n, d, k)
    bad_i = good_i.copy()
    bad_i[k + 1] = bad_i[k]                       # client 1 repeats an index
    for idx in (bad_i, good_i, good_i, bad_i, good_i):
        rec = cuda_records(dev, idx, good_v)
        out = dev.aggregate(4, rec, n, k, d).cpu().numpy()
        assert dev.status() == 0
        ref, st = oracle.non_oblivious(oracle.as_weights(idx, good_v), d, n)
        assert st == 0 and bits_equal(out, ref)


def test_non_oblivious_scatter_sentinel_value(dev, oracle):
    # a value whose bits equal the scatter's empty-slot sentinel (a NaN) takes the
    # in-order sweep, like a repeated index; every other output stays bit-exact
    rng = np.random.default_rng(3)
    n, d, k = 3, 500, 50
    idx, val = rand_sparse(rng, n, d, k)
    val[7] = np.uint32(0xFFFFFFFF).view(np.float32)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(4, rec, n, k, d).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.non_oblivious(oracle.as_weights(idx, val), d, n)
    nan = np.isnan(ref)
    assert st == 0 and nan.sum() == 1 and np.isnan(out[nan]).all()
    assert bits_equal(out[~nan], ref[~nan])


def test_non_oblivious_scatter_rows_reused_across_calls(dev, oracle):
    """The scatter rows are filled with the empty sentinel once per buffer and emptied
    again by each sum: calls of other shapes (the same bytes, another [n][d] layout), the
    baseline sweep writing its dense rows into the same scratch, a repeated index, the
    sentinel value and an out-of-range index in between leave every later call exact."""
    rng = np.random.default_rng(11)
    seq = [(4, 1000, 100, 4, None), (2, 3000, 50, 4, None), (4, 1000, 100, 3, None),
           (4, 1000, 100, 4, None), (3, 700, 60, 4, "repeat"), (3, 700, 60, 4, None),
           (5, 900, 80, 4, "sentinel"), (5, 900, 80, 4, None), (2, 400, 30, 4, "range"),
           (6, 1500, 200, 4, None), (2, 3000, 50, 4, None)]
    for n, d, k, alg, kind in seq:
        idx, val = rand_sparse(rng, n, d, k)
        if kind == "repeat":
            idx[k + 1] = idx[k]
        elif kind == "sentinel":
            val[5] = np.uint32(0xFFFFFFFF).view(np.float32)
        elif kind == "range":
            idx[3] = d + 7
        out = dev.aggregate(alg, cuda_records(dev, idx, val), n, k, d).cpu().numpy()
        if kind == "range":
            assert dev.status() & 0x2
            continue
        assert dev.status() == 0
        ref, st = oracle.non_oblivious(oracle.as_weights(idx, val), d, n)
        ok = ~np.isnan(ref)
        assert st == 0 and bits_equal(out[ok], ref[ok]), (n, d, k, alg, kind)


def test_non_oblivious_index_out_of_range(dev):
    rec = cuda_records(dev, np.array([0, 9], np.uint32), np.ones(2, np.float32))
    dev.aggregate(4, rec, 1, 2, 5)
    assert dev.status() & 0x2


# ---------------------------------------------------------- bitonic ---------
# 2^18: 2^11 tiles + one strided LDS pass; 2^20: 2^12 tiles (512 x 8, direct first pass);
# 2^22: 2^14 tiles + strided passes
@pytest.mark.parametrize("m", [2, 4, 64, 128, 1024, 8192, 1 << 15, 1 << 18, 1 << 20, 1 << 22])
def test_bitonic_idx_network_bit_exact(dev, oracle, m):
    import torch
    rng = np.random.default_rng(m)
    idx = rng.integers(0, max(2, m // 8), m).astype(np.uint32)   # heavy ties
    val = np.arange(m, dtype=np.float32)                          # identity tracking
    rec = cuda_records(dev, idx, val)
    dev.bitonic(rec, 0)
    torch.cuda.synchronize()
    gi, gv = dev.unpack_records(rec.cpu().numpy())
    ref = oracle.bitonic_sort(oracle.as_weights(idx, val))
    assert np.array_equal(gi, ref["idx"]) and bits_equal(gv, ref["val"])


@pytest.mark.parametrize("m", [2, 256, 8192, 1 << 16, 1 << 20, 1 << 22])
def test_keyed_shuffle_bit_exact(dev, oracle, m):
    import torch
    rng = np.random.default_rng(m + 1)
    idx = rng.integers(0, 50, m).astype(np.uint32)
    val = np.arange(m, dtype=np.float32)
    rec = cuda_records(dev, idx, val)
    dev.bitonic(rec, 2, seed=0xC0FFEE)
    torch.cuda.synchronize()
    gi, gv = dev.unpack_records(rec.cpu().numpy())
    ref = oracle.shuffle_keyed(oracle.as_weights(idx, val), 0xC0FFEE)
    assert np.array_equal(gi, ref["idx"]) and bits_equal(gv, ref["val"])


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("m", [1 << 20, 1 << 22, 1 << 24])
def test_bitonic_repeatable(dev, mode, m):
    """The same input through the network three times gives the same bytes (a store
    whose data registers are overwritten too early shows up here as run-to-run noise)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(m + mode)
    base = torch.randint(0, 1 << 20, (m,), generator=g, device="cuda", dtype=torch.int64)
    base = base | (torch.arange(m, device="cuda", dtype=torch.int64) << 32)
    outs = []
    for _ in range(3):
        x = base.clone()
        dev.bitonic(x, mode, seed=11)
        outs.append(x)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_composite_key_sort(dev):
    import torch
    rng = np.random.default_rng(9)
    keys = rng.permutation(1 << 14).astype(np.int64) * 7919 + 3
    t = torch.from_numpy(keys).cuda()
    dev.bitonic(t, 1)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), np.sort(keys))


# ------------------------------------------------- fused producers ---------
@pytest.mark.parametrize("gen", [1, 2])
@pytest.mark.parametrize("nrec,d", [(1_500_001, 200_000), (999_999, 1_200_000), (3_000_000, 100),
                                    (0, 1_500_000), (700_001, 100_000)])
def test_sort_fused_producer_equals_build_then_sort(dev, gen, nrec, d):
    """advanced_init (gen 1) / nips19_build (gen 2) fused into the sort's first pass ==
    the build kernel, then the sort, bit for bit (M >= 2^21, where the fusion applies;
    odd record counts exercise the 16-B load straddling the end of the records)."""
    import torch

    from fltee import _lib as L
    g = torch.Generator(device="cuda").manual_seed(nrec + d)
    idx = torch.randint(0, d + 10, (nrec,), generator=g, device="cuda")
    vbits = torch.randint(0, 1 << 31, (nrec,), generator=g, device="cuda")
    rec = (idx | (vbits << 32)).contiguous()
    if gen == 1:
        tf, key, r = 0, 0, None
        M = 1 << (nrec + d - 1).bit_length()
        ref = dev.advanced_init_range(rec, nrec, d, 0, M)
        dev.bitonic(ref, 0, 0)
    else:
        r, T = dev.laplace_r(d, 50, 100, seed=nrec)
        tf, key = int(T), 0x5EED ^ nrec
        M = 1 << (nrec + d * tf - 1).bit_length()
        ref = dev.nips19_build_range(rec, nrec, r, d, tf, 0, M)
        dev.bitonic(ref, 2, key)
    out = torch.empty(M, dtype=torch.int64, device="cuda")
    st = L.lib().fltee_debug_sort_fused(gen, out.data_ptr(), M, rec.data_ptr(), nrec,
                                        r.data_ptr() if r is not None else None, d, tf, key, None)
    torch.cuda.synchronize()
    assert st == 0
    assert torch.equal(out, ref)


def test_optimized_fused_producer_unaligned_batches(dev):
    """alg 6 batches start at rec + c0*k*8: with k odd every other batch is only 8-B
    aligned, and the fused first pass reads it with 16-B loads (M = 2^21 per batch).
    Same bits as the separate init kernel."""
    import torch

    from fltee import _lib as L
    n, d, k = 2, 2_000_000, 1_500_001
    g = torch.Generator(device="cuda").manual_seed(61)
    idx = torch.cat([torch.randperm(d, generator=g, device="cuda")[:k] for _ in range(n)])
    vals = torch.randn(n * k, generator=g, device="cuda")
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).contiguous()
    try:
        a = dev.aggregate(6, rec, n, k, d, batch=1).cpu().numpy()
        assert dev.status() == 0
        L.lib().fltee_debug_set_fused_init(0)
        b = dev.aggregate(6, rec, n, k, d, batch=1).cpu().numpy()
        assert dev.status() == 0
    finally:
        L.lib().fltee_debug_set_fused_init(1)
    assert bits_equal(a, b)


# -------------------------------------------------------------- fold -------
@pytest.mark.parametrize("n,d,k", [(3, 200, 50), (100, 5000, 500), (40, 70000, 7000)])
def test_fold_bit_exact(dev, oracle, n, d, k):
    import torch
    rng = np.random.default_rng(d)
    idx, val = rand_sparse(rng, n, d, k)
    w = np.concatenate([oracle.as_weights(idx, val),
                        oracle.as_weights(np.arange(d, dtype=np.uint32), np.zeros(d, np.float32))])
    L = len(w)
    M = oracle.next_pow2(L)
    w = np.concatenate([w, oracle.as_weights(np.full(M - L, U32MAX, np.uint32), np.zeros(M - L, np.float32))])
    s = oracle.bitonic_sort(w)
    for fold_len in (L, n * (k // 2) + d):
        src = cuda_records(dev, s["idx"], s["val"])
        dst = torch.empty_like(src)
        st = torch.zeros(1, dtype=torch.int32, device="cuda")
        dev.fold(src, dst, fold_len, n, st)
        torch.cuda.synchronize()
        assert int(st.item()) == 0
        gi, gv = dev.unpack_records(dst.cpu().numpy())
        ref = oracle.fold(s, fold_len)
        assert np.array_equal(gi, ref["idx"]) and bits_equal(gv, ref["val"])


@pytest.mark.parametrize("m,halo,fold_len", [(4096, 8, 4096), (4096, 8, 3000), (1 << 20, 100, 1 << 20),
                                             (1 << 16, 30, 60000)])
def test_fold_long_run(dev, m, halo, fold_len):
    """One run of fold_len records (idx 0, val 1.0) through fltee_fold_device with a halo
    far shorter than the run: no status, exactly one representative of index 0 among
    [0, fold_len) — somewhere inside the run (the patch writes it at a walk's first
    position) — holding the whole run's sum (exact here: integers below 2^24); the rest
    dummies (u32::MAX - p), the positions past fold_len copied."""
    import torch
    idx = np.zeros(m, np.uint32)
    src = cuda_records(dev, idx, np.ones(m, np.float32))
    dst = torch.empty_like(src)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    dev.fold(src, dst, fold_len, halo, st)
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    gi, gv = dev.unpack_records(dst.cpu().numpy())
    reps = np.flatnonzero(gi[:fold_len] == 0)
    assert reps.size == 1 and gv[reps[0]] == np.float32(fold_len)
    others = np.setdiff1d(np.arange(fold_len), reps)
    assert np.array_equal(gi[others], (0xFFFFFFFF - others).astype(np.uint32))
    assert np.array_equal(gi[fold_len:], idx[fold_len:])


# ---------------------------------------------------------- advanced -------
@pytest.mark.parametrize("n,d,k", [(1, 16, 4), (10, 1000, 100), (100, 50890, 5089), (7, 3333, 1)])
def test_advanced_bit_exact(dev, oracle, n, d, k):
    rng = np.random.default_rng(n * 7 + d)
    idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(1, rec, n, k, d).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)


def _advanced_both_ways(dev, rec, n, k, d):
    """advanced with the compaction network (default) and with the enclave's second
    bitonic sort (advanced.rs:106-111)."""
    from fltee import _lib as L
    try:
        a = dev.aggregate(1, rec, n, k, d).cpu().numpy()
        assert dev.status() == 0
        L.lib().fltee_debug_set_advanced_compaction(0)
        b = dev.aggregate(1, rec, n, k, d).cpu().numpy()
        assert dev.status() == 0
    finally:
        L.lib().fltee_debug_set_advanced_compaction(1)
    return a, b


# (n, d, k): compaction levels log2(L - d) = 3 / 14 / 19 / 23 -> 1 / 2 / 3 / 4 passes; the
# last two: a one-band pass padded to the full tile (levels 14-18 of 3.05M records) before a
# final pass without halo rows, and exp5's MLP-MNIST n = 3000 (a final pass without halo)
@pytest.mark.parametrize("n,d,k", [(2, 1_000_000, 3), (1000, 16, 16), (100, 50890, 5089),
                                   (300, 2_000_000, 20_000), (300, 50890, 10_000),
                                   (3000, 50890, 5089)])
def test_advanced_compaction_equals_second_sort(dev, oracle, n, d, k):
    rng = np.random.default_rng(n + d + k)
    idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    a, b = _advanced_both_ways(dev, rec, n, k, d)
    assert bits_equal(a, b)
    if n * k + d <= 600_000:
        ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
        assert st == 0 and bits_equal(a, ref)


# the compaction's last levels as one pass over the output prefix (arrays <= 2^21
# records, k_compact.hip compact_levels): remaining levels 6-10 after the first pass, output
# rows of 1..196 per residue class, rows of 2..16 residues, d below one row (the live-group
# trim), and the streaming fold's converted first pass (n + 1 > 320) in front of it
@pytest.mark.parametrize("n,d,k", [(16, 777, 1500), (64, 100_000, 4000), (3, 5, 70_000),
                                   (400, 5000, 1000), (31, 50_890, 8191)])
def test_advanced_output_prefix_tail_pass(dev, oracle, n, d, k):
    rng = np.random.default_rng(n * 7 + k)
    idx = np.concatenate([np.sort(rng.choice(d, min(k, d), replace=False))
                          if k <= d else rng.integers(0, d, k) for _ in range(n)]).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    # (k > d repeats indices inside a client: runs beyond n + 1, the exact halo)
    out = dev.aggregate(1, rec, n, k, d, fold_halo=n * k + d if k > d else 0).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)


def test_advanced_compaction_out_of_range_and_repeated_indices(dev, oracle):
    # indices >= d fold into their own runs and never reach [0, d); a client's
    # repeated index makes runs longer than n+1 (halo re-run by the ECALL layer,
    # here given directly)
    rng = np.random.default_rng(11)
    n, d, k = 20, 3000, 400
    idx = rng.integers(0, d + 64, n * k).astype(np.uint32)
    val = rng.normal(0, 1, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    from fltee import _lib as L
    try:
        a = dev.aggregate(1, rec, n, k, d, fold_halo=n * k + d).cpu().numpy()
        L.lib().fltee_debug_set_advanced_compaction(0)
        b = dev.aggregate(1, rec, n, k, d, fold_halo=n * k + d).cpu().numpy()
    finally:
        L.lib().fltee_debug_set_advanced_compaction(1)
    assert dev.status() == 0
    ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(a, ref) and bits_equal(b, ref)


def test_advanced_compaction_c5_scale(dev):
    """configs[4] at full size (M = 2^27): compaction network == second bitonic sort,
    bit for bit, and the checksum of the average equals the sum of all values / n."""
    import torch
    n, d, k = 1000, 10_000_000, 100_000
    g = torch.Generator(device="cuda").manual_seed(3)
    vals = torch.randn(n, k, generator=g, device="cuda") * 0.01
    off = torch.randint(0, d, (n, 1), generator=g, device="cuda")
    idx = (off + torch.arange(k, device="cuda").unsqueeze(0)) % d
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
    a, b = _advanced_both_ways(dev, rec, n, k, d)
    assert bits_equal(a, b)
    tot = float(vals.double().sum()) / n
    assert abs(float(np.sum(a, dtype=np.float64)) - tot) < 1e-4 * max(1.0, abs(tot))


def test_advanced_k0_quirk_bit_exact(dev, oracle):
    rng = np.random.default_rng(5)
    n, d = 5, 300
    idx = np.tile(np.arange(d, dtype=np.uint32), n)
    val = rng.normal(0, 1, n * d).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(1, rec, n, d, d, k_req=0, fold_halo=n * d + d).cpu().numpy()
    ref, st = oracle.advanced(0, oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)


@pytest.mark.parametrize("batch", [1, 3, 4, 10])
def test_optimized_alg6_bit_exact(dev, oracle, batch):
    rng = np.random.default_rng(batch)
    n, d, k = 10, 2000, 150
    idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(6, rec, n, k, d, batch=batch).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.client_size_optimized(batch, k, oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)


# ------------------------------------------------------------ nips19 -------
def test_laplace_counts_match_oracle(dev, oracle):
    d, k, n = 44964, 4496, 300
    r, T = dev.laplace_r(d, k, n, seed=77)
    rr, TT = oracle.laplace_r(d, k, n, seed=77)
    assert T == TT
    # ln as (float)ln((double)x) on both sides (k_nips19.hip, fltee_oracle.c): exact
    assert np.array_equal(r.cpu().numpy(), rr)


def test_nips19_bit_exact_vs_oracle(dev, oracle):
    rng = np.random.default_rng(19)
    n, d, k = 12, 3000, 300
    idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(2, rec, n, k, d, seed=1234).cpu().numpy()
    assert dev.status() == 0
    ref, _ = oracle.nips19(k, oracle.as_weights(idx, val), d, n, seed=1234)
    assert bits_equal(out, ref)
    out2 = dev.aggregate(2, rec, n, k, d, seed=1234).cpu().numpy()
    assert bits_equal(out, out2)  # deterministic: no atomics in safe_aggregate


def test_nips19_c4_full_size_bit_exact(dev, oracle):
    """configs[3]: Purchase100 MLP, n = 300 sampled clients, d = 44,964, k = 4,496
    (alpha 0.1): T = 1476.9, d*floor(T) = 66.4 M Laplace dummies, M = 2^27.  Bit-exact
    with the oracle's nips19 (nips19.rs:18-63: the same Laplace counts, keyed shuffle
    network and in-order safe_aggregate; the oracle runs its network on 16 threads,
    which does not change a bit), and within the reassociation bound of the in-order
    (client-order) sum the reference's update_global_weights computes."""
    rng = np.random.default_rng(300)
    n, d, k = 300, 44964, 4496
    idx = np.concatenate([rng.permutation(d)[:k] for _ in range(n)]).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    seed = 0xC4C4
    out = dev.aggregate(2, rec, n, k, d, seed=seed).cpu().numpy()
    assert dev.status() == 0
    w = oracle.as_weights(idx, val)
    oracle.set_threads(16)
    try:
        ref, st = oracle.nips19(k, w, d, n, seed=seed)
    finally:
        oracle.set_threads(1)
    assert st == 0
    assert bits_equal(out, ref)
    inorder, _ = oracle.non_oblivious(w, d, n)
    absum = np.zeros(d, np.float64)
    np.add.at(absum, idx, np.abs(val.astype(np.float64)))
    u = 2.0 ** -24
    bound = 2 * (n - 1) * u * absum / n + 2 * u * np.abs(inorder) + 1e-45
    assert (np.abs(out.astype(np.float64) - inorder) <= bound).all()
    assert np.linalg.norm(out - inorder.astype(np.float64)) <= 1e-6 * np.linalg.norm(inorder)
    # + DP (sigma 1.12, C 1.0; common.rs:56-72): the same aggregate plus N(0, C*sigma)/n
    outdp = dev.aggregate(2, rec, n, k, d, seed=seed, dp=True, sigma=1.12, clipping=1.0).cpu().numpy()
    noise = outdp.astype(np.float64) - out.astype(np.float64)
    sd = 1.12 / n
    assert abs(noise.mean()) < 5 * sd / np.sqrt(d) and abs(noise.std() / sd - 1) < 0.03
    # the same Philox draws as the oracle (f64 log/cos may differ in the last ulp)
    assert np.allclose(outdp, oracle.dp_noise(ref, 1.12, 1.0, n, seed), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("alg,n,d,k", [(1, 100, 50890, 5089), (1, 7, 70000, 3000), (1, 3, 1000, 100),
                                       (2, 12, 3000, 300), (2, 10, 16000, 1000), (4, 40, 1 << 22, 3000),
                                       (1, 1000, 10_000_000, 100_000)])
def test_pad_skip_bit_identical(dev, oracle, alg, n, d, k):
    """The networks skip the stage blocks made of pads alone (level 1, k_bitonic.hip
    stage_steps) and, sorting by key, the pad-only units inside a stage's mixed block
    (level 2, pad_map): the same bits as running them all (level 0), at pad fractions from
    ~0 to ~50 % (advanced C3/C5 shapes, nips19, non_oblivious's composite sort)."""
    from fltee import _lib as L
    rng = np.random.default_rng(n * 7 + d)
    if n * k > 10_000_000:
        idx = ((rng.integers(0, d, n)[:, None] + np.arange(k)[None, :]) % d).reshape(-1).astype(np.uint32)
        val = rng.normal(0, 0.01, n * k).astype(np.float32)
    else:
        idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    outs = []
    for on in (2, 1, 0):
        L.lib().fltee_debug_set_pad_skip(on)
        try:
            outs.append(dev.aggregate(alg, rec, n, k, d, seed=77).cpu().numpy())
        finally:
            L.lib().fltee_debug_set_pad_skip(2)
        assert dev.status() == 0
    assert bits_equal(outs[0], outs[1]) and bits_equal(outs[0], outs[2])
    if n * k <= 2_000_000 and alg != 2:
        ref, st = (oracle.advanced(k, oracle.as_weights(idx, val), d, n) if alg == 1
                   else oracle.non_oblivious(oracle.as_weights(idx, val), d, n))
        assert st == 0 and bits_equal(outs[0], ref)


@pytest.mark.parametrize("alg,n,d,k", [(1, 40, 1_000_000, 60_000), (1, 300, 44964, 14000),
                                       (2, 300, 44964, 4496), (4, 64, 1 << 24, 65536),
                                       (1, 1000, 10_000_000, 100_000)])
def test_swizzled_layout_bit_identical(dev, oracle, alg, n, d, k):
    """The 2^14-tile networks keep the array in the block-swizzled layout between their
    first and last pass (common.h phys): addresses only, the same bits as the plain layout — advanced (mode 0) at 2^22 and at C5's 2^27, nips19's keyed shuffle
    (mode 2, with the selection sink) at C4's 2^27, non_oblivious's composite sort (mode
    1) at 2^22 — and, where the oracle finishes in seconds, the oracle's bits."""
    from fltee import _lib as L
    rng = np.random.default_rng(n * 11 + d)
    if n * k > 10_000_000:
        idx = ((rng.integers(0, d, n)[:, None] + np.arange(k)[None, :]) % d).reshape(-1).astype(np.uint32)
        val = rng.normal(0, 0.01, n * k).astype(np.float32)
    else:
        idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    outs = []
    for on in (1, 0):
        L.lib().fltee_debug_set_swizzle(on)
        try:
            outs.append(dev.aggregate(alg, rec, n, k, d, seed=91).cpu().numpy())
        finally:
            L.lib().fltee_debug_set_swizzle(1)
        assert dev.status() == 0
    for o in outs[1:]:
        assert bits_equal(outs[0], o)
    if n * k <= 4_200_000 and alg == 1:
        ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
        assert st == 0 and bits_equal(outs[0], ref)


@pytest.mark.parametrize("n,d,k,repeat", [(100, 50890, 5089, False), (1000, 200000, 2000, False),
                                          (3, 1000, 1000, False), (30, 3000, 400, True),
                                          (3000, 30000, 16, False), (5000, 20000, 20, False)])
@pytest.mark.parametrize("fused", [True, False])
def test_advanced_fold_fused_into_compaction(dev, oracle, n, d, k, repeat, fused):
    """The fold run inside the compaction's first pass (halo n up to 4096 records; wider
    halos fall back to the separate fold) == the oracle's advanced, bit for bit.  With a
    repeated index (runs longer than the halo n) the default halo n finishes the long
    runs re-associated (no status): bit for bit on every run of <= n + 1 entries, within
    the re-association bound on the others; the run-length halo is exact."""
    from fltee import _lib as L
    rng = np.random.default_rng(n + d)
    idx, val = rand_sparse(rng, n, d, k)
    if repeat:
        idx[:k] = 2200  # client 0 repeats one index k times: a run of ~k records
    rec = cuda_records(dev, idx, val)
    ref, rst = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
    assert rst == 0
    L.lib().fltee_debug_set_fold_compact(1 if fused else 0)
    try:
        out = dev.aggregate(1, rec, n, k, d, fold_halo=(k * n + d) if repeat else 0).cpu().numpy()
        assert dev.status() == 0 and bits_equal(out, ref)
        if repeat:
            from longrun import assert_advanced
            out = dev.aggregate(1, rec, n, k, d).cpu().numpy()
            assert dev.status() == 0
            assert assert_advanced(out, ref, idx, val, d, n) >= 1
    finally:
        L.lib().fltee_debug_set_fold_compact(1)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("adv", ["one_client", "all_one_index", "two_clients_half"])
@pytest.mark.parametrize("alg", [1, 6])
def test_advanced_adversarial_runs_c3_shape(dev, oracle, adv, alg, fused):
    """configs[2]'s shape (n = 100, d = 50890, k = 5089; M = 2^20) with adversarial
    uploads: one client sending one index k times, every record on one
    index (a run of n*k + 1 = 508,901 entries across every tile and lane), two clients
    splitting theirs over two indices.  Fixed cost, no status: every run of <= n + 1
    entries bit for bit against the oracle's advanced (alg 6: its batches of 30), the long
    ones within the re-association bound — through the fused fold + compaction (the
    tiles' look-back carries) and through the streaming fold + patch."""
    from longrun import assert_advanced

    from fltee import _lib as L
    n, d, k = 100, 50890, 5089
    rng = np.random.default_rng(77)
    idx, val = rand_sparse(rng, n, d, k)
    if adv == "one_client":
        idx[:k] = 7
    elif adv == "all_one_index":
        idx[:] = 7
    else:
        idx[k:3 * k] = np.where(np.arange(2 * k) % 2 == 0, 11, 50000).astype(np.uint32)
    rec = cuda_records(dev, idx, val)
    w = oracle.as_weights(idx, val)
    if alg == 1:
        ref, rst = oracle.advanced(k, w, d, n)
    else:
        ref, rst = oracle.client_size_optimized(30, k, w, d, n)
    assert rst == 0
    L.lib().fltee_debug_set_fold_compact(1 if fused else 0)
    try:
        out = dev.aggregate(alg, rec, n, k, d, batch=30 if alg == 6 else 0).cpu().numpy()
        assert dev.status() == 0
    finally:
        L.lib().fltee_debug_set_fold_compact(1)
    assert assert_advanced(out, ref, idx, val, d, n) >= 1


@pytest.mark.parametrize("n,d,k", [(10, 4000, 1000), (10, 8000, 1000), (10, 16000, 1000),
                                   (20, 20000, 2000)])
@pytest.mark.parametrize("fused", [True, False])
def test_nips19_fused_selection_bit_exact(dev, oracle, n, d, k, fused):
    """M = 2^20 (no fusable last pass), 2^21 (2^13 tiles), 2^22 (2^14 tiles), 2^24: the
    selection fused into the shuffle's last pass (fused) and the separate select passes
    give the oracle's nips19 bit for bit."""
    from fltee import _lib as L
    rng = np.random.default_rng(d + n)
    idx, val = rand_sparse(rng, n, d, k)
    rec = cuda_records(dev, idx, val)
    L.lib().fltee_debug_set_nips19_fused_select(1 if fused else 0)
    try:
        out = dev.aggregate(2, rec, n, k, d, seed=99).cpu().numpy()
    finally:
        L.lib().fltee_debug_set_nips19_fused_select(1)
    assert dev.status() == 0
    oracle.set_threads(16)
    try:
        ref, st = oracle.nips19(k, oracle.as_weights(idx, val), d, n, seed=99)
    finally:
        oracle.set_threads(1)
    assert st == 0 and bits_equal(out, ref)


def test_ordered_fold_long_runs(dev, oracle):
    """non_oblivious's stable-sort path (rows too large for scatter rows) with very
    long runs: the wave-per-index fold walks runs of thousands of records in order."""
    rng = np.random.default_rng(8)
    n, d, k = 4, 1 << 23, 60000  # n*d > 64*next_pow2(n*k): the sort path
    idx = np.concatenate([np.where(rng.random(k) < 0.5, 3, rng.integers(0, d, k)) for _ in range(n)]
                         ).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    out = dev.aggregate(4, rec, n, k, d).cpu().numpy()
    assert dev.status() == 0
    ref, st = oracle.non_oblivious(oracle.as_weights(idx, val), d, n)
    assert st == 0 and bits_equal(out, ref)


@pytest.mark.parametrize("d", [1000, 32768, 40000, 44964, 46080, 46081, 100000])
@pytest.mark.parametrize("odd", [False, True])
def test_safe_aggregate_matches_numpy(dev, d, odd):
    """safe_aggregate (common.rs:25-35) on a shuffled-like array: g[idx] += val for idx < d
    in array order (np.add.at in float32 is that sequential sum): bit-exact, for aligned
    and 8-B-aligned (odd start) sources."""
    import torch
    m = (1 << 20) + (1 if odd else 0)
    g = torch.Generator(device="cuda").manual_seed(d)
    idx = torch.randint(0, d + 100, (m,), generator=g, device="cuda")
    vals = torch.randn(m, generator=g, device="cuda")
    buf = (idx | (vals.view(torch.int32).to(torch.int64) << 32))
    src = torch.cat([torch.zeros(1, dtype=torch.int64, device="cuda"), buf])[1:] if odd else buf
    out = dev.safe_aggregate(src, d).cpu().numpy()
    i, v = idx.cpu().numpy(), vals.cpu().numpy()
    ref = np.zeros(d, np.float32)
    sel = i < d
    np.add.at(ref, i[sel], v[sel])
    assert bits_equal(out, ref)


# --------------------------------------------------------------- DP --------
def test_dp_noise_statistics(dev):
    import torch
    n, d = 100, 1 << 20
    rec = torch.from_numpy(dev.pack_records(np.tile(np.arange(d, dtype=np.uint32), 1),
                                            np.zeros(d, np.float32))).cuda()
    out = dev.aggregate(4, rec, 1, d, d, dense=True, dp=True, sigma=1.12, clipping=1.0, seed=5,
                        n_avg=n).cpu().numpy().astype(np.float64)
    sd = 1.12 * 1.0 / n
    assert abs(out.mean()) < 5 * sd / np.sqrt(d)
    assert abs(out.std() / sd - 1) < 0.01
    # 4th moment of a Gaussian: E[z^4] = 3
    assert abs(np.mean((out / sd) ** 4) - 3) < 0.05


def test_dp_noise_matches_reference_distribution(dev):
    # the reference's seeded DP aggregate (update.py:207-224, RandomState(seed+5)) on zero
    # updates, vs the device mechanism (common.rs:56-72): two-sample KS + std
    import torch
    from scipy import stats
    fx = np.load(os.path.join(GOLDEN, "dp_reference.npz"))
    ref = fx["noise"]
    out = torch.zeros(ref.size, dtype=torch.float32, device="cuda")
    dev.dp_noise(out, float(fx["sigma"]), float(fx["clipping"]), int(fx["n"]), seed=99)
    got = out.cpu().numpy()
    assert stats.ks_2samp(got, ref).pvalue > 1e-3
    assert abs(got.std() / ref.std() - 1) < 0.02


def test_dp_noise_matches_oracle_draws(dev, oracle):
    # same Philox stream: device and oracle draw the same noise (f64 log/cos may differ
    # in the last ulp before the f32 rounding)
    import torch
    d, n = 4096, 30
    out = torch.zeros(d, dtype=torch.float32, device="cuda")
    dev.dp_noise(out, 1.12, 1.0, n, seed=4242)
    ref = oracle.dp_noise(np.zeros(d, np.float32), 1.12, 1.0, n, seed=4242)
    assert np.allclose(out.cpu().numpy(), ref, rtol=1e-6, atol=1e-9)


# ------------------------------------------------------------- clip --------
def test_server_side_clip_matches_reference_torch(dev):
    fx = np.load(os.path.join(GOLDEN, "l2clip.npz"))
    d = fx["flat_in"].size
    rec = cuda_records(dev, np.arange(d, dtype=np.uint32), fx["flat_in"])
    out = dev.aggregate(3, rec, 1, d, d, dense=True, clip=True, clipping=float(fx["clipping"]))
    assert np.allclose(out.cpu().numpy(), fx["flat_out"], rtol=1e-6, atol=0)


# -------------------------------------------------------------- AES --------
@pytest.mark.parametrize("name", ["mnist_sparse", "mnist_sparse_clip", "dense_small"])
def test_gpu_decrypt_reference_client_payloads(dev, name):
    import torch
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    ids = fx["client_ids"]
    ct = torch.from_numpy(fx["ciphertext"].copy()).cuda()
    bpc = fx["ciphertext"].size // len(ids)
    out = torch.empty(fx["plaintext"].size // 8, dtype=torch.int64, device="cuda")
    dev.decrypt(ids, ct, bpc, out)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == fx["plaintext"].tobytes()


# The bitsliced kernels take counter windows per wave (the quad kernel 512 blocks: 16
# quads x 32 slices; the byte-per-lane kernel 128: 4 x 16 lanes x 32 slices): slices
# shorter than a window, ending one record into a window, a half last block (odd record
# count), several clients per window row, unaligned slices (bpc % 8 != 0) and 32-bit
# client ids — through each kernel (variant 1 quad, 2 byte-per-lane, 0 by size).
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("n,bpc", [(1, 8), (3, 24), (2, 16 * 2048), (2, 16 * 2048 + 8),
                                   (5, 16 * 2048 * 2 - 8), (7, 40712), (4, 8 * 5089 + 3),
                                   (3, 16 * 4096 + 13), (2, 16 * 128 + 8), (9, 16 * 127)])
def test_gpu_decrypt_bitsliced_windows(dev, oracle, n, bpc, variant):
    from fltee import _lib
    _lib.lib().fltee_debug_set_aes_variant(variant)
    try:
        _decrypt_windows_case(dev, oracle, n, bpc)
    finally:
        _lib.lib().fltee_debug_set_aes_variant(0)


def _decrypt_windows_case(dev, oracle, n, bpc):
    import torch
    rng = np.random.default_rng(bpc * 31 + n)
    ids = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ids[0] = 0xFFFFFFFF
    ct = rng.integers(0, 256, n * bpc, dtype=np.uint8)
    rpc = bpc // 8
    want = b"".join(oracle.aes128_ctr(oracle.session_key(int(ids[c])),
                                      ct[c * bpc:(c + 1) * bpc].tobytes())[:rpc * 8]
                    for c in range(n))
    out = torch.full((n * rpc,), -1, dtype=torch.int64, device="cuda")
    dev.decrypt(ids, torch.from_numpy(ct).cuda(), bpc, out)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == want


# ------------------------------------------------------- full size NS ------
def test_headline_shape_100x1M_bit_exact(dev):
    import torch
    n, d = 100, 1_000_000
    g = torch.Generator(device="cuda").manual_seed(13)
    vals = torch.randn(n, d, generator=g, device="cuda") * 0.01
    idx = torch.arange(d, device="cuda", dtype=torch.int64).repeat(n, 1)
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
    out = dev.aggregate(3, rec, n, d, d, dense=True).cpu().numpy()
    assert dev.status() == 0
    v = vals.cpu().numpy()
    ref = np.sum(v, axis=0, dtype=np.float32) * np.float32(np.float32(1) / np.float32(n))
    assert bits_equal(out, ref)
    # bench checksum (benchmark.rs:226-239)
    assert abs(float(out.astype(np.float64).sum()) - float(v.astype(np.float64).sum()) / n) < 1e-3


# ------------------------------------------------- multi-GPU building blocks ----
def test_parallel_paths_single_rank(dev, oracle):
    """fltee.parallel with the real kernels (world = 1): column split + dense kernel, and
    client-range `advanced` partials combined by fltee_sum_rows_device (alg-6 order)."""
    import torch

    from fltee import parallel as P
    rng = np.random.default_rng(77)
    n, d = 6, 1001
    dense = rng.normal(0, 0.01, (n, d)).astype(np.float32)
    rec, lo, hi = P.split_dense_columns(torch.from_numpy(dense).cuda(), 1, 0)
    full = P.param_sharded_dense(rec, n, hi - lo, d, 1, 0).cpu().numpy()
    ref = oracle.baseline(oracle.as_weights(np.tile(np.arange(d, dtype=np.uint32), n),
                                            dense.reshape(-1)), d, n)
    assert bits_equal(full, ref)
    nc, dk, k = 8, 700, 40
    idx, val = rand_sparse(rng, nc, dk, k)
    out = P.client_sharded_advanced(cuda_records(dev, idx, val), nc, k, dk, nc, 1, 0)
    ref, st = oracle.client_size_optimized(nc, k, oracle.as_weights(idx, val), dk, nc)
    assert st == 0 and bits_equal(out.cpu().numpy(), ref)
    # two "ranks" emulated in one process: partials of clients [0,4) and [4,8) summed in order
    parts = [dev.aggregate(1, cuda_records(dev, idx[c0 * k:c1 * k], val[c0 * k:c1 * k]),
                           c1 - c0, k, dk, no_average=True) for c0, c1 in ((0, 4), (4, 8))]
    coef = float(np.float32(1) / np.float32(nc))
    got = dev.sum_rows(torch.stack(parts), coef).cpu().numpy()
    ref, st = oracle.client_size_optimized(4, k, oracle.as_weights(idx, val), dk, nc)
    assert st == 0 and bits_equal(got, ref)


@pytest.mark.parametrize("alg,n,d,k", [(2, 300, 44964, 4496), (2, 12, 3000, 300), (4, 2, 2_000_000, 100),
                                       (4, 3, 1 << 24, 50000)])
def test_radix_order_equals_composite_sort(dev, alg, n, d, k):
    """The ordered folds' stable order by (idx, position) from the radix sort by idx
    (k_radix.hip, the default) == the composite-key bitonic sort, bit for bit: nips19's
    selected list (C4 shape and a small one) and non_oblivious's sparse fallback (repeated
    indices across clients, runs in upload order)."""
    from fltee import _lib as L
    rng = np.random.default_rng(n * 31 + d)
    idx = rng.integers(0, d, n * k).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    rec = cuda_records(dev, idx, val)
    outs = []
    try:
        for on in (1, 0):
            L.lib().fltee_debug_set_radix_order(on)
            outs.append(dev.aggregate(alg, rec, n, k, d, seed=91).cpu().numpy())
            assert dev.status() == 0
    finally:
        L.lib().fltee_debug_set_radix_order(1)
    assert bits_equal(outs[0], outs[1])

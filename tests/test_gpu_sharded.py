"""GPU parity of position-range sharded `advanced` (SURVEY §8e Option B): the HIP
range pieces driven by fltee.parallel.index_sharded_advanced with every range on one
GPU (VirtualRanks: the exchanges are device copies) must reproduce the oracle's
single-process network permutation and `advanced` output bit for bit."""
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


def case(seed, n, d, k, idx_hi=None):
    rng = np.random.default_rng(seed)
    if idx_hi is None:
        idx = np.concatenate([rng.choice(d, k, replace=False) for _ in range(n)]).astype(np.uint32)
    else:
        idx = rng.integers(0, idx_hi, n * k).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    return idx, val


def init_chunks(dev, rec, nrec, d, world, M):
    C = M // world
    return {r: dev.advanced_init_range(rec[r * C:] if r * C < nrec else rec, nrec, d, r * C, C)
            for r in range(world)}


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("world,m", [(2, 1 << 10), (4, 1 << 15), (8, 1 << 20), (8, 512), (2, 1 << 22)])
def test_distributed_network_equals_single_sort(dev, oracle, world, m, mode):
    """Range sorts + exchanges + range merges == the reference network on all M (mode 0:
    advanced's sort; mode 2: nips19's keyed shuffle, pairwise exchanges)."""
    import torch

    from fltee.parallel import DeviceRangeOps, VirtualRanks, distributed_network
    rng = np.random.default_rng(m + world)
    idx = rng.integers(0, max(2, m // 8), m).astype(np.uint32)   # heavy ties
    val = np.arange(m, dtype=np.float32)                          # identity tracking
    full = torch.from_numpy(dev.pack_records(idx, val)).cuda()
    C = m // world
    chunks = {r: full[r * C:(r + 1) * C].clone() for r in range(world)}
    out = distributed_network(chunks, world, m, DeviceRangeOps(), VirtualRanks(world), mode=mode,
                              seed=0xC0FFEE, exchange="pairwise")
    got = torch.cat([out[r] for r in range(world)]).cpu().numpy()
    gi, gv = dev.unpack_records(got)
    w = oracle.as_weights(idx, val)
    ref = oracle.bitonic_sort(w) if mode == 0 else oracle.shuffle_keyed(w, 0xC0FFEE)
    assert np.array_equal(gi, ref["idx"]) and np.array_equal(gv.view(np.uint32), ref["val"].view(np.uint32))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_index_sharded_nips19_matches_single_gpu(dev, world):
    """nips19 by position range == fltee_aggregate_device(nips19) with the same seed:
    same Laplace counts, same shuffle, each index's entries added in shuffled order on
    both: bit-identical."""
    import torch

    from fltee.parallel import VirtualRanks, index_sharded_nips19
    n, d, k, seed = 30, 4000, 400, 1234
    idx, val = case(7 + world, n, d, k)
    rec = torch.from_numpy(dev.pack_records(idx, val)).cuda()
    single = dev.aggregate(2, rec, n, k, d, seed=seed).cpu().numpy()
    assert dev.status() == 0
    r, T = dev.laplace_r(d, k, n, seed)
    tf = int(T)
    nrec = n * k
    M = 1 << (nrec + d * tf - 1).bit_length()
    C = M // world
    chunks = {q: dev.nips19_build_range(rec[q * C:] if q * C < nrec else rec, nrec, r, d, tf,
                                        q * C, C) for q in range(world)}
    out = index_sharded_nips19(chunks, world, M, n, d, seed, comm=VirtualRanks(world),
                               valid=nrec + d * tf).cpu().numpy()
    assert np.array_equal(out.view(np.uint32), single.view(np.uint32))


@pytest.mark.parametrize("exchange", ["transpose", "pairwise"])
@pytest.mark.parametrize("world,n,d,k,idx_hi", [(2, 20, 3000, 400, None), (4, 20, 3000, 400, None),
                                                (8, 4, 100, 50, None), (8, 100, 50890, 5089, None),
                                                (2, 7, 3333, 1, None), (4, 20, 3000, 400, 64),
                                                (4, 30, 2000, 300, 2100)])
def test_index_sharded_advanced_bit_exact(dev, oracle, world, n, d, k, idx_hi, exchange):
    """idx_hi = 64: runs far longer than n + 1, across the ranges — finished through the
    ranges' totals and the patch (round 6): within the re-association bound of the
    oracle, the rest bit for bit; 2100 > d: indices outside [0, d) fold into their own
    runs and never reach the output."""
    import torch

    from longrun import assert_advanced

    from fltee.parallel import VirtualRanks, index_sharded_advanced
    idx, val = case(world * 1000 + n + d, n, d, k, idx_hi)
    rec = torch.from_numpy(dev.pack_records(idx, val)).cuda()
    M = oracle.next_pow2(n * k + d)
    chunks = init_chunks(dev, rec, n * k, d, world, M)
    out = index_sharded_advanced(chunks, world, M, n, k, d, comm=VirtualRanks(world),
                                 exchange=exchange)
    ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
    assert st == 0
    got = out.cpu().numpy()
    nlong = assert_advanced(got, ref, idx, val, d, n)
    assert (nlong > 0) == (idx_hi == 64)


def test_index_sharded_matches_single_gpu_at_scale(dev):
    """configs[2]-like shape at 2^21: sharded x4 == fltee_aggregate_device(advanced)."""
    import torch

    from fltee.parallel import VirtualRanks, index_sharded_advanced
    n, d, k = 300, 50890, 5089
    idx, val = case(5, n, d, k)
    rec = torch.from_numpy(dev.pack_records(idx, val)).cuda()
    single = dev.aggregate(1, rec, n, k, d).cpu().numpy()
    assert dev.status() == 0
    M = 1 << (n * k + d - 1).bit_length()
    out = index_sharded_advanced(init_chunks(dev, rec, n * k, d, 4, M), 4, M, n, k, d,
                                 comm=VirtualRanks(4)).cpu().numpy()
    assert np.array_equal(out.view(np.uint32), single.view(np.uint32))


@pytest.mark.parametrize("m,d,hi", [(1, 10, 20), (777, 50, 80), (40000, 3000, 3100), (5000, 100, 100),
                                    (5000, 100, 90000),
                                    # the counting sort's shapes (k_radix.hip): one pass of 3
                                    # bits; one index (a run over every wave); a tile plus one;
                                    # 17 key bits (3 passes of 6); 24 bits over mostly gaps
                                    (100000, 5, 5), (4097, 1, 1), (2049, 3000, 3000),
                                    (70000, 65536, 65536), (300000, 10_000_000, 10_000_000)])
def test_select_and_ordered_list_match_numpy(dev, m, d, hi):
    """fltee_select_device (entries with idx < d, position order) and
    fltee_ordered_list_device (in-order f32 sums x coef) == numpy, bit for bit; hi = d:
    nothing selected; the per-range lists concatenated reproduce one range's sums."""
    import torch

    from range_ops_np import NumpyRangeOps
    rng = np.random.default_rng(m + d)
    idx = rng.integers(0, hi, m).astype(np.uint32)
    val = rng.normal(0, 1, m).astype(np.float32)
    x = torch.from_numpy(dev.pack_records(idx, val).view(np.int64)).cuda()
    lst = dev.select(x, d)
    ref = NumpyRangeOps().select(x.cpu(), d)
    assert np.array_equal(lst.cpu().numpy(), ref.numpy())
    coef = float(np.float32(1.0) / np.float32(7))
    out = dev.ordered_list(lst, d, coef).cpu().numpy()
    want = NumpyRangeOps().ordered(ref, d, coef).numpy()
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))
    parts = [dev.select(x[a:b], d) for a, b in ((0, m // 3), (m // 3, m // 2), (m // 2, m))]
    out2 = dev.ordered_list(torch.cat(parts), d, coef).cpu().numpy()
    assert np.array_equal(out2.view(np.uint32), out.view(np.uint32))

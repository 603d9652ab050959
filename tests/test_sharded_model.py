"""Option B (position-range sharded `advanced`) on CPU: the driver in
fltee.parallel with numpy stand-ins for the range pieces, every range in one process
(VirtualRanks) — must equal the oracle's single-process `advanced` bit for bit."""
import numpy as np
import pytest
import torch

from longrun import assert_advanced
from range_ops_np import NumpyRangeOps, init_range


def case(seed, n, d, k, idx_hi=None):
    rng = np.random.default_rng(seed)
    if idx_hi is None:
        idx = np.concatenate([rng.choice(d, k, replace=False) for _ in range(n)]).astype(np.uint32)
    else:
        idx = rng.integers(0, idx_hi, n * k).astype(np.uint32)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    return idx, val


@pytest.mark.parametrize("exchange", ["transpose", "pairwise"])
@pytest.mark.parametrize("world,n,d,k,idx_hi", [(1, 5, 200, 30, None), (2, 5, 200, 30, None),
                                                (4, 6, 300, 20, None), (8, 4, 100, 50, None),
                                                (4, 10, 150, 40, 40), (2, 7, 333, 1, None),
                                                (4, 10, 150, 40, 1), (8, 30, 100, 60, 3)])
def test_virtual_ranks_match_oracle(oracle, world, n, d, k, idx_hi, exchange):
    from fltee.parallel import VirtualRanks, index_sharded_advanced
    idx, val = case(world * 100 + n, n, d, k, idx_hi)
    M = oracle.next_pow2(n * k + d)
    C = M // world
    chunks = {r: init_range(idx, val, d, r * C, C) for r in range(world)}
    out = index_sharded_advanced(chunks, world, M, n, k, d, ops=NumpyRangeOps(),
                                 comm=VirtualRanks(world), exchange=exchange)
    ref, st = oracle.advanced(k, oracle.as_weights(idx, val), d, n)
    assert st == 0
    # bit for bit; idx_hi: runs of more than n + 1 entries re-associated (longrun.py)
    nlong = assert_advanced(out.numpy(), ref, idx, val, d, n)
    assert idx_hi is not None or nlong == 0


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_virtual_keyed_shuffle_network(oracle, world):
    """The distributed network in mode 2 (nips19's keyed shuffle) == the oracle's
    single-array shuffle, bit for bit."""
    from fltee.parallel import VirtualRanks, distributed_network
    rng = np.random.default_rng(world)
    m = 1024
    idx = rng.integers(0, 50, m).astype(np.uint32)
    val = np.arange(m, dtype=np.float32)
    w = oracle.as_weights(idx, val)
    full = torch.from_numpy(w.view(np.int64).copy())
    C = m // world
    chunks = {r: full[r * C:(r + 1) * C].clone() for r in range(world)}
    out = distributed_network(chunks, world, m, NumpyRangeOps(), VirtualRanks(world), mode=2,
                              seed=0xC0FFEE)
    got = torch.cat([out[r] for r in range(world)]).numpy()
    ref = oracle.shuffle_keyed(w, 0xC0FFEE)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))

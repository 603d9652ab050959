"""CPU model of the oblivious compaction network that replaces advanced's second sort
(fl-tee_amd/csrc/k_compact.hip; advanced.rs:106-111).

After the fold the array is sorted by index with one representative per index
0..d-1 (the run sum) and dummies / pads / indices >= d elsewhere.  The second
bitonic sort's [0, d) prefix is then the idx < d records in position order.  This
restates the network level by level in numpy (no tiling) and checks, on random
folded arrays, that (a) selected records never collide and (b) the prefix equals
what a sort produces.  The GPU tests check the tiled kernel against the bitonic
sort and the oracle.
"""
import numpy as np
import pytest

U32MAX = 0xFFFFFFFF


def compaction_network(keys, vals, d):
    L = keys.size
    nlev = int(L - d).bit_length() if L > d else 0
    k, v = keys.astype(np.int64).copy(), vals.copy()
    pos = np.arange(L, dtype=np.int64)
    for j in range(nlev):
        sel = k < d
        move = sel & (((pos - k) >> j) & 1).astype(bool)
        stay = sel & ~move
        nk = np.full(L, U32MAX, np.int64)
        nv = np.zeros(L, np.float32)
        nk[stay], nv[stay] = k[stay], v[stay]
        dst = pos[move] - (1 << j)
        # no selected record lands on a staying one or on another mover
        assert not np.any(stay[dst]) and np.unique(dst).size == dst.size
        nk[dst], nv[dst] = k[move], v[move]
        k, v = nk, nv
    return k[:d], v[:d]


def folded_array(rng, d, extra, oob):
    """d representatives (idx 0..d-1, ascending), `extra` dummies (U32MAX - p) and
    `oob` representatives of indices >= d, interleaved like a folded sorted array."""
    L = d + extra + oob
    sel_pos = np.sort(rng.choice(d + extra, d, replace=False))
    keys = np.empty(L, np.int64)
    is_rep = np.zeros(d + extra, bool)
    is_rep[sel_pos] = True
    keys[: d + extra][is_rep] = np.arange(d)
    keys[: d + extra][~is_rep] = U32MAX - np.nonzero(~is_rep)[0]
    keys[d + extra:] = d + np.arange(oob)  # sorted after every idx < d
    vals = rng.normal(0, 1, L).astype(np.float32)
    return keys, vals


@pytest.mark.parametrize("d,extra,oob", [(1, 0, 0), (1, 1, 0), (5, 37, 3), (100, 3000, 0),
                                         (4096, 4096 * 7 + 11, 100), (1000, 1, 5)])
def test_network_equals_sort_prefix(d, extra, oob):
    rng = np.random.default_rng(d * 31 + extra)
    keys, vals = folded_array(rng, d, extra, oob)
    ck, cv = compaction_network(keys, vals, d)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(ck, keys[order][:d])
    assert np.array_equal(cv.view(np.uint32), vals[order][:d].view(np.uint32))


def test_network_adversarial_gaps():
    # every representative as far right as possible, then as far left as possible
    for d, extra in [(7, 57), (64, 1000)]:
        L = d + extra
        keys = np.concatenate([U32MAX - np.arange(extra), np.arange(d)]).astype(np.int64)
        vals = np.arange(L, dtype=np.float32)
        ck, cv = compaction_network(keys, vals, d)
        assert np.array_equal(ck, np.arange(d)) and np.array_equal(cv, vals[extra:])
        keys = np.concatenate([np.arange(d), U32MAX - np.arange(extra)]).astype(np.int64)
        ck, cv = compaction_network(keys, vals, d)
        assert np.array_equal(ck, np.arange(d)) and np.array_equal(cv, vals[:d])

"""CPU model of the client producers' ordering (k_client.hip) against the reference's
zero_except_top_k_weights output (tests/golden/client_producer.npz, utils.py:327-354)."""
import os

import numpy as np

from conftest import GOLDEN


def composite_keys(flat):
    """The kernel's key: ((0x7FFFFFFF - |v| bits) << 32) | idx, ascending = reference order."""
    a = flat.astype(np.float32).view(np.uint32) & np.uint32(0x7FFFFFFF)
    return ((np.uint64(0x7FFFFFFF) - a.astype(np.uint64)) << np.uint64(32)) | np.arange(
        flat.size, dtype=np.uint64)


def test_composite_key_order_is_reference_topk():
    fx = np.load(os.path.join(GOLDEN, "client_producer.npz"))
    k = int(fx["k"])
    for c, flat in enumerate(fx["flats"]):
        order = np.argsort(composite_keys(flat), kind="stable")[:k]
        assert np.array_equal(order.astype(np.uint32), fx["topk"][c])
        # and the plain records are (idx, flat[idx]) in that order
        rec = fx["plain"].reshape(len(fx["flats"]), k, 8)[c]
        assert np.array_equal(rec[:, :4].copy().view("<u4").ravel(), order)
        assert np.array_equal(rec[:, 4:].copy().view("<f4").ravel().view(np.uint32),
                              flat[order].view(np.uint32))


def test_fixture_has_boundary_ties():
    fx = np.load(os.path.join(GOLDEN, "client_producer.npz"))
    k = int(fx["k"])
    a = np.abs(fx["flats"][2])
    kth = np.sort(a)[::-1][k - 1]
    assert (a == kth).sum() > 1 and (a > kth).sum() < k  # the cut falls inside a tie group

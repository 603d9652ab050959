"""configs[4] (C5) at full size against the oracle: `advanced` over n = 1000 clients x
k = 100,000 records into d = 10,000,000 (L = n*k + d = 110 M, M = 2^27 entries).

* the device path (`fltee_aggregate_device`) bit for bit against the oracle's
  `fo_advanced` (advanced.rs:39-113: padded array, bitonic sort, fold, second sort,
  first d run sums x 1f32/n), the oracle's comparator networks on 16 threads (each
  step's compare-exchanges are independent: the same bits as one thread);
* the same output within the reassociation bound of the in-order (client-order) sum
  the reference's update_global_weights computes (update.py:173-184);
* the ECALL (lib.rs:221-423) on a one-GPU eid and on an 8-rank eid
  (fltee_device_init_multi, every range on this GPU: the position-range network with
  its all-to-all exchanges, the halo fold, per-range compaction and the reduce of
  group.hip) — the same bits as the device path.
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

N, D, K = 1000, 10_000_000, 100_000
U = 2.0 ** -24


@pytest.fixture(scope="module")
def c5():
    """Every client uploads k distinct indices (a run from a random offset, mod d: the
    shape top-k uploads have), values N(0, 0.01)."""
    rng = np.random.default_rng(0xC5)
    off = rng.integers(0, D, N, dtype=np.int64)
    idx = ((off[:, None] + np.arange(K, dtype=np.int64)[None, :]) % D).reshape(-1).astype(np.uint32)
    val = rng.normal(0, 0.01, N * K).astype(np.float32)
    return idx, val


@pytest.fixture(scope="module")
def device_out(c5):
    import torch

    from fltee import device as dev
    torch.cuda.init()
    idx, val = c5
    rec = torch.from_numpy(dev.pack_records(idx, val)).cuda()
    out = dev.aggregate(1, rec, N, K, D).cpu().numpy()
    assert dev.status() == 0
    del rec
    torch.cuda.empty_cache()
    return out


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def test_advanced_c5_full_size_bit_exact_vs_oracle(c5, device_out, oracle):
    idx, val = c5
    w = oracle.as_weights(idx, val)
    oracle.set_threads(16)
    try:
        ref, st = oracle.advanced(K, w, D, N)
    finally:
        oracle.set_threads(1)
    assert st == 0
    assert np.array_equal(bits(device_out), bits(ref))
    # vs the in-order client sum (update_global_weights): a reassociation of the same values
    inorder, st = oracle.non_oblivious(w, D, N)
    assert st == 0
    absum = np.zeros(D, np.float64)
    np.add.at(absum, idx, np.abs(val.astype(np.float64)))
    o = device_out.astype(np.float64)
    bound = 2 * (N - 1) * U * absum / N + 2 * U * np.abs(inorder) + 1e-45
    assert (np.abs(o - inorder) <= bound).all()
    assert np.linalg.norm(o - inorder) <= 1e-6 * np.linalg.norm(inorder)


def _ecall(E, ids, enc, fl_id):
    from fltee.ecalls import set_debug_seed
    set_debug_seed(0xC5C5)
    try:
        assert E.ecall_fl_init(fl_id, ids, D, K, 1.12, 1.0, 0.1, 1.0, 1, 0, 0) == (0, 0)
        assert E.ecall_start_round(fl_id, 0, len(ids))[:2] == (0, 0)
        st, rv, out, times = E.ecall_secure_aggregation(fl_id, 0, ids, enc, D, K, 1)
    finally:
        set_debug_seed(0)
    assert (st, rv) == (0, 0)
    assert np.isfinite(times).all()
    return out


def test_advanced_c5_ecall_one_gpu_and_8_rank_eid(c5, device_out, oracle):
    idx, val = c5
    ids = np.arange(20000, 20000 + N, dtype=np.uint32)
    w = oracle.as_weights(idx, val).reshape(N, K)
    enc = oracle.encrypt_clients(ids, [w[i].tobytes() for i in range(N)])
    del w
    from fltee.ecalls import Enclave
    one = Enclave(0)
    try:
        out1 = _ecall(one, ids, enc, 7701)
    finally:
        one.destroy()
    assert np.array_equal(bits(out1), bits(device_out))
    grp = Enclave([0] * 8)
    try:
        assert grp.device_count() == 8
        out8 = _ecall(grp, ids, enc, 7702)
    finally:
        grp.destroy()
    assert np.array_equal(bits(out8), bits(device_out))


@pytest.mark.parametrize("adv", ["one_client", "all_one_index"])
def test_advanced_c5_adversarial_runs(c5, adv):
    """configs[4] at full size with adversarial uploads: client 0 sending
    one index k = 100,000 times, and all n*k = 10^8 records on one index (one run over
    ~50,000 fold lanes).  One fixed-cost pass, no status; every index within the bound
    any f32 left fold of its run obeys against the exact (float64) sum — the full-size
    property check (the oracle's network at 2^27 per case would take minutes)."""
    import torch

    from longrun import assert_near_exact

    from fltee import device as dev
    idx, val = c5
    idx = idx.copy()
    if adv == "one_client":
        idx[:K] = 7
    else:
        idx[:] = 7
    rec = torch.from_numpy(dev.pack_records(idx, val)).cuda()
    out = dev.aggregate(1, rec, N, K, D).cpu().numpy()
    assert dev.status() == 0
    del rec
    torch.cuda.empty_cache()
    assert_near_exact(out, idx, val, D, N)

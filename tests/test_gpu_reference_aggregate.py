"""GPU parity against the REFERENCE's own aggregate (not only the oracle).

Inputs: the payloads the reference's client code produced (tests/golden/
ref_aggregate.npz, made by tests/golden/make_fixtures.py), encrypted with the
oracle's AES (pinned to the reference's encryption.cpp) and sent through the C-ABI
ECALLs of libfltee_agg.so exactly as server.rs would.  Expected: the reference's
in-order aggregator src/update.py:173-184 update_global_weights on the same
updates.  Criteria (tests/refcheck.py): in-order algorithms (non_oblivious,
baseline, path_oram) bit-exact at power-of-two n and within 1 ulp otherwise (the
reference divides, the enclave multiplies by 1f32/n); advanced, nips19 and alg 6
(sort / shuffle / batch order) within 1e-6 relative plus the per-index
reassociation bound.  Every GPU result is also checked bit for bit against the
oracle's restated enclave on the same inputs where the oracle is cheap enough.
"""
import numpy as np
import pytest

import refcheck as R
from conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

SEED = 0xA66


@pytest.fixture(scope="module")
def enclave():
    import torch
    torch.cuda.init()
    from fltee.ecalls import Enclave
    e = Enclave(0)
    yield e
    e.destroy()


_enc_cache = {}


def payload(oracle, c):
    if c["name"] not in _enc_cache:
        w = R.records(c).reshape(c["n"], c["k"])
        _enc_cache[c["name"]] = oracle.encrypt_clients(
            c["client_ids"], [w[i].tobytes() for i in range(c["n"])])
    return _enc_cache[c["name"]]


_fl = [1000]


def round0(E, c, alg):
    _fl[0] += 1
    fl = _fl[0]
    ids = c["client_ids"]
    assert E.ecall_fl_init(fl, ids, c["d"], c["k"], 1.12, 1.0, 0.1, 1.0, alg, 0, 0) == (0, 0)
    st, rv, _ = E.ecall_start_round(fl, 0, len(ids))
    assert (st, rv) == (0, 0)
    return fl


IN_ORDER = [(name, alg) for name in R.cases() for alg in (3, 4, 5)]


@pytest.mark.parametrize("name,alg", IN_ORDER)
def test_ecall_in_order_algs_match_reference(enclave, oracle, name, alg):
    c = R.case(name)
    fl = round0(enclave, c, alg)
    st, rv, out, times = enclave.ecall_secure_aggregation(fl, 0, c["client_ids"], payload(oracle, c),
                                                          c["d"], c["k"], alg)
    assert (st, rv) == (0, 0) and np.isfinite(times).all()
    R.assert_in_order_exact(out, c)


@pytest.mark.parametrize("name", [c for c in R.cases() if c.startswith("sparse")])
def test_ecall_advanced_matches_reference(enclave, oracle, name):
    c = R.case(name)
    fl = round0(enclave, c, 1)
    st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, c["client_ids"], payload(oracle, c),
                                                      c["d"], c["k"], 1)
    assert (st, rv) == (0, 0)
    R.assert_reassociated(out, c)
    ref, ost = oracle.advanced(c["k"], R.records(c), c["d"], c["n"])
    assert ost == 0 and np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("name,batch", [("sparse_n4", 4), ("sparse_n32", 5), ("sparse_n30", 30),
                                        ("sparse_n100", 33)])
def test_ecall_alg6_matches_reference(enclave, oracle, name, batch):
    c = R.case(name)
    fl = round0(enclave, c, 6)
    st, rv, out, _ = enclave.ecall_client_size_optimized_secure_aggregation(
        fl, 0, batch, c["client_ids"], payload(oracle, c), c["d"], c["k"], 6)
    assert (st, rv) == (0, 0)
    R.assert_reassociated(out, c)
    ref, ost = oracle.client_size_optimized(batch, c["k"], R.records(c), c["d"], c["n"])
    assert ost == 0 and np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("name", ["sparse_n4", "sparse_n32", "sparse_n30", "sparse_n100", "dense_n30"])
def test_ecall_nips19_matches_reference(enclave, oracle, name):
    """Full-size nips19 (request k = the payload's k: d*floor(T) Laplace dummies, up to
    M = 2^27 at n = 100) through the ECALL, vs the reference's in-order sum."""
    c = R.case(name)
    fl = round0(enclave, c, 2)
    st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, c["client_ids"], payload(oracle, c),
                                                      c["d"], c["k"], 2)
    assert (st, rv) == (0, 0)
    R.assert_reassociated(out, c)


@pytest.mark.parametrize("name", ["sparse_n4", "sparse_n30", "dense_n32"])
def test_device_nips19_bit_exact_vs_oracle_and_close_to_reference(oracle, name):
    """The device entry point with a fixed seed: bit-exact with the oracle's nips19
    (same Laplace counts, same keyed shuffle, in-order safe_aggregate) and within the
    reassociation bound of the reference's aggregate.  k_req = 16 keeps the oracle's
    padded array small; every real record is still summed."""
    import torch

    from fltee import device as D
    c = R.case(name)
    w = R.records(c)
    rec = torch.from_numpy(np.ascontiguousarray(w).view(np.int64).copy()).cuda()
    out = D.aggregate(2, rec, c["n"], c["k"], c["d"], seed=SEED, k_req=16).cpu().numpy()
    assert D.status() == 0
    oracle.set_threads(16)
    try:
        ref, st = oracle.nips19(16, w, c["d"], c["n"], seed=SEED)
    finally:
        oracle.set_threads(1)
    assert st == 0
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    R.assert_reassociated(out, c)


# ---- configs[3]'s full shape: Purchase100 x 300 clients (ref_aggregate_cfg.npz; the
# payloads are rebuilt from seeds and checked against the reference client's bytes) ----

def cfg_payload(oracle, c):
    if c["name"] not in _enc_cache:
        w = R.records(c).reshape(c["n"], c["k"])
        _enc_cache[c["name"]] = oracle.encrypt_clients(
            c["client_ids"], [w[i].tobytes() for i in range(c["n"])])
    return _enc_cache[c["name"]]


CFG_IN_ORDER = [("purchase100_sparse_n300", 3), ("purchase100_sparse_n300", 4),
                ("purchase100_sparse_n300", 5), ("purchase100_dense_n300", 3),
                ("purchase100_dense_n300", 4)]


@pytest.mark.parametrize("name,alg", CFG_IN_ORDER)
def test_cfg_ecall_in_order_algs_match_reference(enclave, oracle, name, alg):
    """baseline / non_oblivious / path_oram through the ECALL at configs[3]'s size vs
    the reference's update_global_weights: within 1 ulp (n = 300)."""
    c = R.cfg_case(name)
    fl = round0(enclave, c, alg)
    st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, c["client_ids"], cfg_payload(oracle, c),
                                                      c["d"], c["k"], alg)
    assert (st, rv) == (0, 0)
    R.assert_in_order_exact(out, c)


def test_cfg_ecall_advanced_matches_reference(enclave, oracle):
    """advanced (M = 2^21) at configs[3]'s size: within the reassociation bound of the
    reference's aggregate, and bit for bit the oracle's network."""
    c = R.cfg_case("purchase100_sparse_n300")
    fl = round0(enclave, c, 1)
    st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, c["client_ids"], cfg_payload(oracle, c),
                                                      c["d"], c["k"], 1)
    assert (st, rv) == (0, 0)
    R.assert_reassociated(out, c)
    ref, ost = oracle.advanced(c["k"], R.records(c), c["d"], c["n"])
    assert ost == 0 and np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_cfg_ecall_nips19_and_alg6_match_reference(enclave, oracle):
    """nips19 at configs[3]'s full size (request k = 4,496: the C4 shuffle, M = 2^27) and
    alg 6 in batches of 64, vs the reference's aggregate."""
    c = R.cfg_case("purchase100_sparse_n300")
    fl = round0(enclave, c, 2)
    st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, c["client_ids"], cfg_payload(oracle, c),
                                                      c["d"], c["k"], 2)
    assert (st, rv) == (0, 0)
    R.assert_reassociated(out, c)
    fl = round0(enclave, c, 6)
    st, rv, out, _ = enclave.ecall_client_size_optimized_secure_aggregation(
        fl, 0, 64, c["client_ids"], cfg_payload(oracle, c), c["d"], c["k"], 6)
    assert (st, rv) == (0, 0)
    R.assert_reassociated(out, c)
    ref, ost = oracle.client_size_optimized(64, c["k"], R.records(c), c["d"], c["n"])
    assert ost == 0 and np.array_equal(out.view(np.uint32), ref.view(np.uint32))

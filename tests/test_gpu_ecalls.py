"""The four ECALLs through libfltee_agg.so vs the oracle's restated enclave.

Inputs are the reference Python client's own payloads (tests/golden/).  Both
state machines run from the same debug seed, so client sampling, nips19 and DP
draws line up call for call.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

SEED = 0x5EED


@pytest.fixture(scope="module")
def enclave():
    import torch
    torch.cuda.init()
    from fltee.ecalls import Enclave
    e = Enclave(0)
    yield e
    e.destroy()


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32),
                          np.asarray(b, np.float32).view(np.uint32))


def run_round(E, ids, d, k, alg, enc, fl_id, ratio=1.0, dp=0, sigma=1.12, clipping=1.0):
    st, rv = E.ecall_fl_init(fl_id, ids, d, k, sigma, clipping, 0.1, ratio, alg, 0, dp)
    assert (st, rv) == (0, 0)
    sample = int(np.float32(len(ids)) * np.float32(ratio))
    st, rv, sampled = E.ecall_start_round(fl_id, 0, sample)
    assert (st, rv) == (0, 0)
    return sampled


@pytest.mark.parametrize("alg", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("name", ["mnist_sparse", "mnist_sparse_clip"])
def test_secure_aggregation_matches_oracle(enclave, oracle, alg, name):
    from fltee.ecalls import set_debug_seed
    fx = load(name)
    ids, d, k = fx["client_ids"], int(fx["d"]), int(fx["k"])
    enc = fx["ciphertext"].tobytes()
    set_debug_seed(SEED)
    O = oracle.OracleEnclave(seed=SEED)
    fl = 100 + alg
    sampled = run_round(enclave, ids, d, k, alg, enc, fl)
    assert O.fl_init(fl, ids, d, k, 1.12, 1.0, 0.1, 1.0, alg) == 0
    st, osampled = O.start_round(fl, 0, len(ids))
    assert np.array_equal(sampled, osampled)
    st, rv, out, times = enclave.ecall_secure_aggregation(fl, 0, ids, enc, d, k, alg)
    assert (st, rv) == (0, 0)
    assert np.isfinite(times).all() and (times >= 0).all()
    ost, ref, _ = O.secure_aggregation(fl, 0, ids, enc, d, k, alg)
    assert ost == 0
    assert bits_equal(out, ref)
    # round advanced: the same round is now rejected (lib.rs:241-243,421)
    st, rv, out2, _ = enclave.ecall_secure_aggregation(fl, 0, ids, enc, d, k, alg)
    assert (st, rv) == (0, 2) and not out2.any()
    set_debug_seed(0)


def test_dense_payload_baseline(enclave, oracle):
    fx = load("dense_small")
    ids, d = fx["client_ids"], int(fx["d"])
    run_round(enclave, ids, d, 0, 3, None, 7)
    st, rv, out, _ = enclave.ecall_secure_aggregation(7, 0, ids, fx["ciphertext"].tobytes(), d, 0, 3)
    assert (st, rv) == (0, 0) and bits_equal(out, fx["oracle_baseline"])


@pytest.mark.parametrize("batch", [1, 3, 4])
def test_client_size_optimized_matches_oracle(enclave, oracle, batch):
    fx = load("mnist_sparse")
    ids, d, k = fx["client_ids"], int(fx["d"]), int(fx["k"])
    enc = fx["ciphertext"].tobytes()
    O = oracle.OracleEnclave(seed=1)
    fl = 200 + batch
    run_round(enclave, ids, d, k, 6, enc, fl)
    O.fl_init(fl, ids, d, k, 1.12, 1.0, 0.1, 1.0, 6)
    O.start_round(fl, 0, len(ids))
    st, rv, out, times = enclave.ecall_client_size_optimized_secure_aggregation(fl, 0, batch, ids, enc, d, k, 6)
    assert (st, rv) == (0, 0) and times[2] == 0
    ost, ref, _ = O.client_size_optimized_secure_aggregation(fl, 0, batch, ids, enc, d, k, 6)
    assert ost == 0 and bits_equal(out, ref)


def test_dp_noise_through_ecall(enclave, oracle):
    fx = load("mnist_sparse")
    ids, d, k = fx["client_ids"], int(fx["d"]), int(fx["k"])
    enc = fx["ciphertext"].tobytes()
    run_round(enclave, ids, d, k, 4, enc, 300, dp=1)
    st, rv, out, _ = enclave.ecall_secure_aggregation(300, 0, ids, enc, d, k, 4)
    assert (st, rv) == (0, 0)
    noise = out.astype(np.float64) - fx["oracle_non_oblivious"].astype(np.float64)
    sd = 1.12 * 1.0 / len(ids)  # common.rs:67-71: N(0, C*sigma) / n
    assert abs(noise.mean()) < 5 * sd / np.sqrt(d)
    assert abs(noise.std() / sd - 1) < 0.03


def test_sampling_matches_oracle(enclave, oracle):
    from fltee.ecalls import set_debug_seed
    ids = np.arange(1000, 1100, dtype=np.uint32)
    set_debug_seed(77)
    O = oracle.OracleEnclave(seed=77)
    O.fl_init(5, ids, 10, 1, 1.0, 1.0, 0.1, 0.3, 4)
    st, rv = enclave.ecall_fl_init(5, ids, 10, 1, 1.0, 1.0, 0.1, 0.3, 4, 0, 0)
    assert (st, rv) == (0, 0)
    st, rv, s = enclave.ecall_start_round(5, 0, 30)
    ost, os_ = O.start_round(5, 0, 30)
    assert (st, rv, ost) == (0, 0, 0) and np.array_equal(s, os_)
    assert enclave.ecall_start_round(5, 0, 29)[1] == 2          # lib.rs:200-203
    set_debug_seed(0)


def test_error_paths(enclave):
    from fltee import _lib as L
    fx = load("mnist_sparse")
    ids, d, k = fx["client_ids"], int(fx["d"]), int(fx["k"])
    enc = fx["ciphertext"].tobytes()
    run_round(enclave, ids, d, k, 4, enc, 400)
    st, rv, out, times = enclave.ecall_secure_aggregation(999, 0, ids, enc, d, k, 4)
    assert (st, rv) == (0, L.ERROR_UNEXPECTED) and not out.any()   # unknown fl_id
    st, rv, out, _ = enclave.ecall_secure_aggregation(400, 0, ids, enc, d, k, 1)
    assert rv == L.ERROR_INVALID_PARAMETER and not out.any()      # alg mismatch
    st, rv, _, _ = enclave.ecall_secure_aggregation(400, 0, ids[::-1][:3], enc, d, k, 4)
    assert rv == L.ERROR_INVALID_PARAMETER                         # id set mismatch
    from fltee.ecalls import Enclave
    bogus = Enclave.__new__(Enclave)
    bogus.lib, bogus.eid = enclave.lib, 12345
    assert bogus.ecall_secure_aggregation(400, 1, ids, enc, d, k, 4)[0] == L.ERROR_INVALID_ENCLAVE_ID
    run_round(enclave, ids, d, k, 7, enc, 401)
    assert enclave.ecall_secure_aggregation(401, 0, ids, enc, d, k, 7)[1] == L.ERROR_INVALID_PARAMETER


def _encrypt(oracle, ids, recs):
    return oracle.encrypt_clients(ids, [r.tobytes() for r in recs])


def test_advanced_long_run_is_folded(enclave, oracle):
    """advanced's fold runs once with halo n — fixed cost.  A client repeating one index k
    times makes a run of ~k entries, more than the n + 1 that distinct indices allow: the
    ECALL returns the reference's aggregate (round 6: no 0x2), every run of <= n + 1
    entries bit for bit and the long one within the re-association bound, for alg 1 and
    alg 6.  A repeated index that keeps every run within n + 1 entries is exact."""
    from longrun import assert_advanced
    from fltee import _lib as L
    from fltee.ecalls import set_debug_seed
    n = 30
    rng = np.random.default_rng(5)
    ids = np.arange(500, 500 + n, dtype=np.uint32)
    for k, d, reps, want in ((4000, 4000, 4000, 0), (1000, 4000, 3, 0)):
        recs = []
        for c in range(n):
            w = np.zeros(k, dtype=oracle.WEIGHT)
            w["idx"] = rng.permutation(d)[:k]
            if c == 3:
                w["idx"][:reps] = 7  # client 3 repeats index 7 `reps` times
            w["val"] = rng.normal(0, 0.01, k).astype(np.float32)
            recs.append(w)
        enc = _encrypt(oracle, ids, recs)
        for alg, fl in ((1, 610 + reps), (6, 620 + reps)):
            set_debug_seed(SEED)
            O = oracle.OracleEnclave(seed=SEED)
            run_round(enclave, ids, d, k, alg, enc, fl)
            O.fl_init(fl, ids, d, k, 1.12, 1.0, 0.1, 1.0, alg)
            O.start_round(fl, 0, n)
            if alg == 1:
                st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, ids, enc, d, k, alg)
                ost, ref, _ = O.secure_aggregation(fl, 0, ids, enc, d, k, alg)
            else:
                st, rv, out, _ = enclave.ecall_client_size_optimized_secure_aggregation(
                    fl, 0, 7, ids, enc, d, k, alg)
                ost, ref, _ = O.client_size_optimized_secure_aggregation(fl, 0, 7, ids, enc, d, k, alg)
            assert (st, rv, ost) == (0, want, 0)
            allw = np.concatenate(recs)
            nlong = assert_advanced(out, ref, allw["idx"], allw["val"], d, n)
            assert (nlong > 0) == (reps > n)
    set_debug_seed(0)


@pytest.mark.parametrize("k_req", [0, 1, 50, 300])
def test_nips19_uses_request_k(enclave, oracle, k_req):
    """nips19.rs:38 takes T (and the Laplace scale) from the request's
    num_of_sparse_parameters, not from the payload's record count; fl_main.py sends
    dense uploads with k = 0 (no --alpha), where T = 0 and no dummies are added."""
    from fltee.ecalls import set_debug_seed
    n, d, rpc = 6, 2000, 300
    rng = np.random.default_rng(k_req)
    ids = np.arange(40, 40 + n, dtype=np.uint32)
    recs = []
    for _ in range(n):
        w = np.zeros(rpc, dtype=oracle.WEIGHT)
        w["idx"] = rng.permutation(d)[:rpc]
        w["val"] = rng.normal(0, 0.01, rpc).astype(np.float32)
        recs.append(w)
    enc = _encrypt(oracle, ids, recs)
    fl = 700 + k_req
    set_debug_seed(SEED)
    O = oracle.OracleEnclave(seed=SEED)
    run_round(enclave, ids, d, k_req, 2, enc, fl)
    O.fl_init(fl, ids, d, k_req, 1.12, 1.0, 0.1, 1.0, 2)
    O.start_round(fl, 0, n)
    st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, ids, enc, d, k_req, 2)
    ost, ref, _ = O.secure_aggregation(fl, 0, ids, enc, d, k_req, 2)
    assert (st, rv, ost) == (0, 0, 0)
    assert bits_equal(out, ref)
    set_debug_seed(0)


@pytest.mark.parametrize("alg", [1, 6])
def test_repeated_small_calls_of_one_shape(enclave, oracle, alg):
    """Small `advanced` / alg-6 ECALLs of one shape, back to back, through the zero-copy
    staging (ecalls.hip staged_ecall): every call must read its own payload — new values,
    a rejected upload (status word) in between, another shape in between — and match the
    oracle bit for bit."""
    rng = np.random.default_rng(90 + alg)
    d, k = 3000, 40

    def payload(ids, kk, dup=False):
        plain = []
        for _ in ids:
            idx = rng.choice(d, kk, replace=False).astype(np.uint32)
            if dup:
                idx[1] = idx[0]  # a repeated index: a run of n + 2 entries is possible
            plain.append(oracle.as_weights(idx, rng.normal(0, 1, kk).astype(np.float32)).tobytes())
        return oracle.encrypt_clients(ids, plain)

    def call(fl, ids, kk, enc):
        O = oracle.OracleEnclave(seed=SEED)
        run_round(enclave, ids, d, kk, alg, enc, fl)
        O.fl_init(fl, ids, d, kk, 1.12, 1.0, 0.1, 1.0, alg)
        O.start_round(fl, 0, len(ids))
        if alg == 6:
            st, rv, out, _ = enclave.ecall_client_size_optimized_secure_aggregation(
                fl, 0, 2, ids, enc, d, kk, 6)
            ost, ref, _ = O.client_size_optimized_secure_aggregation(fl, 0, 2, ids, enc, d, kk, 6)
        else:
            st, rv, out, _ = enclave.ecall_secure_aggregation(fl, 0, ids, enc, d, kk, alg)
            ost, ref, _ = O.secure_aggregation(fl, 0, ids, enc, d, kk, alg)
        return st, rv, out, ost, ref

    ids = np.array([11, 12, 13, 14, 15], np.uint32)
    fl = 900 + 20 * alg
    for r in range(6):
        kk = 25 if r == 3 else k  # round 3: another shape, then back
        dup = r == 4 and len(ids) == 1
        st, rv, out, ost, ref = call(fl + r, ids, kk, payload(ids, kk, dup))
        assert st == 0 and rv == ost == 0, (r, rv, ost)
        assert bits_equal(out, ref), r
    # a run longer than n + 1 (round 6: folded, no 0x2), and the next call of the shape is
    # bit for bit again
    one = np.array([21], np.uint32)
    for r in range(3):
        st, rv, out, ost, ref = call(fl + 10 + r, one, k, payload(one, k, dup=(r == 1)))
        assert st == 0 and rv == ost == 0
        if r != 1:
            assert bits_equal(out, ref)
        else:
            assert np.allclose(out, ref, rtol=1e-5, atol=1e-9)

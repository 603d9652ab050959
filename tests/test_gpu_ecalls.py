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
    if alg == 2:  # nips19: atomics-based scatter, fp32 tolerance
        assert np.abs(out - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max()) * 5
    else:
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

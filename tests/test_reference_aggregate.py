"""Pin the oracle's aggregation ARITHMETIC to the reference's own aggregator.

tests/golden/ref_aggregate.npz holds client payloads produced by the reference's
client code (zero_except_top_k_weights + serialize_sparse / serialize_dense,
utils.py) and the output of the reference's in-order aggregator on the same
updates, src/update.py:173-184 update_global_weights (tests/golden/make_fixtures.py).
The criteria are in tests/refcheck.py: in-order algorithms are bit-exact at
power-of-two n and within 1 ulp otherwise (torch.div vs the enclave's x * (1f32/n),
common.rs:14-19); reassociating ones are within 1e-6 relative.
The GPU side of the same checks is tests/test_gpu_reference_aggregate.py.
"""
import numpy as np
import pytest

import refcheck as R

SPARSE = [c for c in R.cases() if c.startswith("sparse")]
DENSE = [c for c in R.cases() if c.startswith("dense")]


def test_fixture_is_the_reference_sum():
    # the fixture's divisor identity: for n a power of two, torch.div(x, n) == x * (1/n)
    for name in R.cases():
        c = R.case(name)
        assert c["ref_avg"].shape == (c["d"],) and np.isfinite(c["ref_avg"]).all()
        assert len(c["plaintext"]) == c["n"] * c["k"] * 8
        w = R.records(c)
        assert (w["idx"] < c["d"]).all()
        if c["dense"]:
            assert np.array_equal(w["idx"].reshape(c["n"], c["d"]),
                                  np.tile(np.arange(c["d"], dtype=np.uint32), (c["n"], 1)))


@pytest.mark.parametrize("name", R.cases())
def test_oracle_non_oblivious_matches_reference(oracle, name):
    c = R.case(name)
    g, st = oracle.non_oblivious(R.records(c), c["d"], c["n"])
    assert st == 0
    R.assert_in_order_exact(g, c)


@pytest.mark.parametrize("name", ["sparse_n4", "sparse_n30", "sparse_n32", "dense_n4", "dense_n30"])
def test_oracle_baseline_and_path_oram_match_reference(oracle, name):
    c = R.case(name)
    w = R.records(c)
    R.assert_in_order_exact(oracle.baseline(w, c["d"], c["n"]), c)
    g, st = oracle.path_oram(w, c["d"], c["n"])
    assert st == 0
    R.assert_in_order_exact(g, c)


@pytest.mark.parametrize("name", ["sparse_n4", "sparse_n30", "sparse_n32", "sparse_n100"])
def test_oracle_advanced_matches_reference(oracle, name):
    c = R.case(name)
    g, st = oracle.advanced(c["k"], R.records(c), c["d"], c["n"])
    assert st == 0
    R.assert_reassociated(g, c)


@pytest.mark.parametrize("name,batch", [("sparse_n4", 4), ("sparse_n32", 32), ("sparse_n30", 7),
                                        ("sparse_n32", 5)])
def test_oracle_alg6_matches_reference(oracle, name, batch):
    c = R.case(name)
    g, st = oracle.client_size_optimized(batch, c["k"], R.records(c), c["d"], c["n"])
    assert st == 0
    R.assert_reassociated(g, c)


@pytest.mark.parametrize("name", ["sparse_n4", "sparse_n32", "dense_n30"])
def test_oracle_nips19_matches_reference(oracle, name):
    # nips19 adds d*floor(T) zero-valued dummies and sums in shuffled order; the
    # request's k only sets T and the Laplace scale (nips19.rs:38), so a small
    # k_req keeps the padded array CPU-sized while every real record is summed
    c = R.case(name)
    oracle.set_threads(8)
    try:
        g, st = oracle.nips19(16, R.records(c), c["d"], c["n"], seed=0xC0FFEE)
    finally:
        oracle.set_threads(1)
    assert st == 0
    R.assert_reassociated(g, c)


def test_oracle_ecall_matches_reference(oracle):
    """The whole ECALL (decrypt with the session keys, dispatch, average) on the
    reference's payloads, encrypted with the AES pinned to encryption.cpp."""
    c = R.case("sparse_n32")
    ids, d, k = c["client_ids"], c["d"], c["k"]
    w = R.records(c).reshape(c["n"], k)
    enc = oracle.encrypt_clients(ids, [w[i].tobytes() for i in range(c["n"])])
    for alg in (4, 1):
        E = oracle.OracleEnclave(seed=9)
        assert E.fl_init(50 + alg, ids, d, k, 1.12, 1.0, 0.1, 1.0, alg) == 0
        assert E.start_round(50 + alg, 0, len(ids))[0] == 0
        st, out, _ = E.secure_aggregation(50 + alg, 0, ids, enc, d, k, alg)
        assert st == 0
        if alg == 4:
            R.assert_in_order_exact(out, c)
        else:
            R.assert_reassociated(out, c)


# ---- configs[3]'s full shape (Purchase100, 300 clients): ref_aggregate_cfg.npz ------

CFG = R.cfg_cases()


@pytest.mark.parametrize("name", CFG)
def test_cfg_payload_regenerates_the_reference_bytes(name):
    """The records the tests rebuild from the stored seeds are byte for byte the
    payloads the reference's client code serialised (sha256 in the fixture)."""
    c = R.cfg_case(name)  # asserts the sha256
    w = R.records(c)
    assert w.size == c["n"] * c["k"] and (w["idx"] < c["d"]).all()
    assert c["ref_avg"].shape == (c["d"],) and np.isfinite(c["ref_avg"]).all()


@pytest.mark.parametrize("name", CFG)
def test_cfg_oracle_in_order_matches_reference(oracle, name):
    """non_oblivious (and, sparse, baseline's o_update sweep) at the full configuration
    vs update_global_weights (n = 300: within 1 ulp — torch.div vs x * (1f32/n)).  The
    dense baseline is the same in-order sum; its oracle sweep takes a minute here, so
    the GPU test covers it (test_gpu_reference_aggregate.py)."""
    c = R.cfg_case(name)
    w = R.records(c)
    g, st = oracle.non_oblivious(w, c["d"], c["n"])
    assert st == 0
    R.assert_in_order_exact(g, c)
    if not c["dense"]:
        R.assert_in_order_exact(oracle.baseline(w, c["d"], c["n"]), c)


def test_cfg_oracle_advanced_matches_reference(oracle):
    """advanced at configs[3]'s size (M = 2^21 network) vs the reference's aggregate."""
    c = R.cfg_case("purchase100_sparse_n300")
    g, st = oracle.advanced(c["k"], R.records(c), c["d"], c["n"])
    assert st == 0
    R.assert_reassociated(g, c)

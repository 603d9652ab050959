"""A multi-GPU enclave id behind the unchanged ECALL ABI (fltee_device_init_multi,
group.hip): every algorithm returns the same bits as the single-GPU eid.

On the one-GPU test box the ranks are virtual (the same device repeated: every range
on one GPU, the exchanges device copies) — the sharding, the distributed network,
the halo fold, the reduce and the gathers all run exactly as on W GPUs; only the
transport differs.  [0] alone opens a one-rank RCCL communicator, so the RCCL
calls themselves (ncclCommInitAll, grouped send/recv, ncclReduce) run too.  The
8-GPU RCCL path is measured by bench.py's multi-GPU run (extra.c_abi_multi_gpu).
"""
import numpy as np
import pytest

import refcheck as R
from conftest import gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

SEED = 0x6A0


@pytest.fixture(scope="module")
def enclaves():
    import torch
    torch.cuda.init()
    from fltee.ecalls import Enclave
    es = {1: Enclave(0), "rccl1": Enclave([0])}
    for w in (2, 4, 8):
        es[w] = Enclave([0] * w)
    yield es
    for e in es.values():
        e.destroy()


_fl = [5000]


def run(E, c, alg, enc, batch=None, k=None):
    from fltee.ecalls import set_debug_seed
    _fl[0] += 1
    fl = _fl[0]
    ids = c["client_ids"]
    k = c["k"] if k is None else k
    set_debug_seed(SEED)
    assert E.ecall_fl_init(fl, ids, c["d"], k, 1.12, 1.0, 0.1, 1.0, alg, 0, 0) == (0, 0)
    assert E.ecall_start_round(fl, 0, len(ids))[:2] == (0, 0)
    if alg == 6:
        st, rv, out, times = E.ecall_client_size_optimized_secure_aggregation(
            fl, 0, batch, ids, enc, c["d"], k, 6)
    else:
        st, rv, out, times = E.ecall_secure_aggregation(fl, 0, ids, enc, c["d"], k, alg)
    set_debug_seed(0)
    assert (st, rv) == (0, 0)
    assert np.isfinite(times).all()
    return out


_enc = {}


def payload(oracle, c):
    if c["name"] not in _enc:
        w = R.records(c).reshape(c["n"], c["k"])
        _enc[c["name"]] = oracle.encrypt_clients(c["client_ids"], [w[i].tobytes() for i in range(c["n"])])
    return _enc[c["name"]]


def test_device_counts(enclaves):
    assert enclaves[1].device_count() == 1 and enclaves["rccl1"].device_count() == 1
    assert [enclaves[w].device_count() for w in (2, 4, 8)] == [2, 4, 8]


def test_bad_device_lists_are_refused():
    from fltee.ecalls import Enclave
    for devs in ([], [0, 0, 0], [0] * 128):
        with pytest.raises(RuntimeError):
            Enclave(devs)


CASES = [("dense_n30", 3), ("dense_n30", 4), ("dense_n32", 5), ("sparse_n32", 4), ("sparse_n30", 3),
         ("sparse_n32", 1), ("sparse_n100", 1), ("sparse_n4", 1), ("sparse_n32", 2), ("sparse_n100", 2),
         ("dense_n4", 2)]


@pytest.mark.parametrize("name,alg", CASES)
@pytest.mark.parametrize("w", [2, 4, 8, "rccl1"])
def test_group_ecall_bit_identical_to_one_gpu(enclaves, oracle, name, alg, w):
    c = R.case(name)
    enc = payload(oracle, c)
    one = run(enclaves[1], c, alg, enc)
    grp = run(enclaves[w], c, alg, enc)
    assert np.array_equal(one.view(np.uint32), grp.view(np.uint32))
    if alg in (3, 4, 5):
        R.assert_in_order_exact(grp, c)
    else:
        R.assert_reassociated(grp, c)


@pytest.mark.parametrize("name,batch", [("sparse_n32", 5), ("sparse_n30", 30), ("sparse_n100", 7)])
@pytest.mark.parametrize("w", [2, 8, "rccl1"])
def test_group_alg6_bit_identical_to_one_gpu(enclaves, oracle, name, batch, w):
    c = R.case(name)
    enc = payload(oracle, c)
    one = run(enclaves[1], c, 6, enc, batch=batch)
    grp = run(enclaves[w], c, 6, enc, batch=batch)
    assert np.array_equal(one.view(np.uint32), grp.view(np.uint32))
    R.assert_reassociated(grp, c)


def test_group_advanced_long_run_and_k_quirk(enclaves, oracle):
    """A client repeating one index (a run of more than n + 1 entries): every eid folds it
    in one fixed-cost pass (round 6) — the long run crossing the position ranges finished
    through the ranges' totals (group.hip) — every other index bit for bit against the
    oracle, the long one within the re-association bound; the k=0 dense quirk
    (advanced.rs:70, the root path) equals the single-GPU result."""
    from longrun import assert_advanced

    from fltee.ecalls import set_debug_seed
    rng = np.random.default_rng(3)
    n, k, d = 16, 3000, 3000
    ids = np.arange(900, 900 + n, dtype=np.uint32)
    recs, plain = [], []
    for i in range(n):
        w = np.zeros(k, dtype=oracle.WEIGHT)
        w["idx"] = rng.permutation(d)[:k]
        w["val"] = rng.normal(0, 0.01, k).astype(np.float32)
        plain.append(w.copy())
        if i == 5:
            w["idx"] = 11
        recs.append(w)
    enc = oracle.encrypt_clients(ids, [r.tobytes() for r in recs])
    allw = np.concatenate(recs)
    ref, rst = oracle.advanced(k, allw, d, n)
    assert rst == 0
    for w in (1, 2, 8):
        E = enclaves[w]
        _fl[0] += 1
        set_debug_seed(SEED)
        assert E.ecall_fl_init(_fl[0], ids, d, k, 1.12, 1.0, 0.1, 1.0, 1, 0, 0) == (0, 0)
        assert E.ecall_start_round(_fl[0], 0, n)[:2] == (0, 0)
        st, rv, out, _ = E.ecall_secure_aggregation(_fl[0], 0, ids, enc, d, k, 1)
        set_debug_seed(0)
        assert (st, rv) == (0, 0)
        assert assert_advanced(out, ref, allw["idx"], allw["val"], d, n) == 1, w
    enc0 = oracle.encrypt_clients(ids, [r.tobytes() for r in plain])
    c = dict(client_ids=ids, d=d, k=k, n=n, name="quirk")
    one0 = run(enclaves[1], c, 1, enc0, k=0)
    assert np.array_equal(one0.view(np.uint32), run(enclaves[4], c, 1, enc0, k=0).view(np.uint32))


@pytest.mark.parametrize("alg", [1, 2, 4])
def test_group_ragged_payload(enclaves, oracle, alg):
    """Client slices of 8*k + 3 bytes (lib.rs:305-306 floors bytes and records per
    client): every GPU loads whole clients that cover its range at byte offsets that are
    not record-aligned; the result equals the single-GPU eid's."""
    rng = np.random.default_rng(alg)
    n, k, d = 10, 301, 1000
    ids = np.arange(70, 70 + n, dtype=np.uint32)
    slices = []
    for i in ids:
        w = np.zeros(k, dtype=oracle.WEIGHT)
        w["idx"] = rng.permutation(d)[:k]
        w["val"] = rng.normal(0, 0.01, k).astype(np.float32)
        slices.append(oracle.aes128_ctr(oracle.session_key(int(i)), w.tobytes() + b"\x01\x02\x03"))
    enc = b"".join(slices)
    c = dict(client_ids=ids, d=d, k=k, n=n, name=f"ragged{alg}")
    one = run(enclaves[1], c, alg, enc)
    for w in (2, 8):
        assert np.array_equal(one.view(np.uint32), run(enclaves[w], c, alg, enc).view(np.uint32))


@pytest.mark.parametrize("w", [2, 8])
def test_group_nips19_declined_shape_same_seed(enclaves, oracle, w):
    """A nips19 shape the group declines (C = M / W < 64: group.hip's fallback to the root
    path) draws the call's seed once, like one GPU: under fltee_debug_set_seed both eids
    give the same Laplace counts, shuffle and DP-free sum."""
    rng = np.random.default_rng(w)
    n, k, d = 4, 4, 16
    ids = np.arange(300, 300 + n, dtype=np.uint32)
    recs = []
    for _ in range(n):
        r = np.zeros(k, dtype=oracle.WEIGHT)
        r["idx"] = rng.permutation(d)[:k]
        r["val"] = rng.normal(0, 0.01, k).astype(np.float32)
        recs.append(r)
    enc = oracle.encrypt_clients(ids, [r.tobytes() for r in recs])
    c = dict(client_ids=ids, d=d, k=k, n=n, name=f"tiny_nips19_{w}")
    one = run(enclaves[1], c, 2, enc)
    assert np.array_equal(one.view(np.uint32), run(enclaves[w], c, 2, enc).view(np.uint32))


def test_group_exact_runs_policy_and_dense_order(enclaves, oracle):
    """fltee_set_advanced_exact_runs(1): the long run above is folded exactly on every eid
    (the one-GPU sequential walk; the group path declines) and alg 6 likewise — the
    oracle's advanced bit for bit.  Dense-sized uploads out of position: every flat alg
    reruns them sparse on the root (baseline / path_oram through the composite-key
    network's ordered fold), the reference's in-order sum bit for bit on every eid."""
    from fltee import _lib as L
    from fltee.ecalls import set_advanced_exact_runs, set_debug_seed
    rng = np.random.default_rng(5)
    n, k, d = 6, 700, 900
    ids = np.arange(600, 600 + n, dtype=np.uint32)
    recs = []
    for i in range(n):
        w = np.zeros(k, dtype=oracle.WEIGHT)
        w["idx"] = rng.permutation(d)[:k]
        w["val"] = rng.normal(0, 0.01, k).astype(np.float32)
        if i == 2:
            w["idx"][:300] = 11  # a run of ~300 entries
        recs.append(w)
    allw = np.concatenate(recs)
    enc = oracle.encrypt_clients(ids, [r.tobytes() for r in recs])
    ref, st = oracle.advanced(k, allw, d, n)
    assert st == 0
    set_advanced_exact_runs(True)
    try:
        for w in (1, 2, 8):
            c = dict(client_ids=ids, d=d, k=k, n=n, name=f"exact{w}")
            out = run(enclaves[w], c, 1, enc)
            assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), w
            o6 = run(enclaves[w], c, 6, enc, batch=4)
            assert np.array_equal(o6.view(np.uint32), run(enclaves[1], c, 6, enc, batch=4).view(np.uint32))
    finally:
        set_advanced_exact_runs(False)
    # dense-sized, out of position
    d2 = 640
    plain = []
    for _ in ids:
        p = np.zeros(d2, dtype=oracle.WEIGHT)
        p["idx"] = rng.permutation(d2)
        p["val"] = rng.normal(0, 1, d2).astype(np.float32)
        plain.append(p)
    enc2 = oracle.encrypt_clients(ids, [p.tobytes() for p in plain])
    exp, _ = oracle.non_oblivious(np.concatenate(plain), d2, n)
    for w in (1, 2, 8):
        for alg in (3, 4, 5):
            E = enclaves[w]
            _fl[0] += 1
            set_debug_seed(SEED)
            assert E.ecall_fl_init(_fl[0], ids, d2, d2, 1.12, 1.0, 0.1, 1.0, alg, 0, 0) == (0, 0)
            assert E.ecall_start_round(_fl[0], 0, n)[:2] == (0, 0)
            st, rv, out, _ = E.ecall_secure_aggregation(_fl[0], 0, ids, enc2, d2, d2, alg)
            set_debug_seed(0)
            # every flat alg reruns it sparse on the root: the in-order sum, bit for bit
            assert (st, rv) == (0, 0) and np.array_equal(out.view(np.uint32), exp.view(np.uint32)), (w, alg)

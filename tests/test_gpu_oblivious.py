"""Obliviousness of the launch trace (DESIGN §7's "public sizes only").

Everything the host side of the library does on the GPU — every kernel launch (its call
site, grid, block, LDS), every copy / memset (kind, bytes), every host synchronisation,
every RCCL send / receive / reduce and the launch-side bytes of the streaming passes —
goes through the trace wrappers of csrc/common.h (tests/test_abi.py rejects a raw call in
csrc/).  For two inputs with the same public sizes (alg, n, k, d, seed) and different
data — random uploads, and adversarial ones (one client sending one index k times, every
record on one index) — the traces must be identical, line for line: the launch sequence
reveals the sizes only.  Covered: advanced (fused and streaming folds), alg 6, baseline
sparse (sweep; dense-sized: the composite-key network), path_oram as the tree, the dense
algs, nips19 (every record's idx < d, so its selected count — the one data-sized quantity,
DESIGN §7 — is the same), and the ECALLs (small staged path, large pipelined path).
Documented exceptions (not tested here): non_oblivious (not oblivious in the reference
either) and nips19's selected count.  Each shape runs once untraced first (the scratch
allocations of a first call are not part of the steady-state trace)."""
import ctypes

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


def _lib():
    from fltee import _lib as L
    lib = L.lib()
    lib.fltee_debug_trace.argtypes = [ctypes.c_int]
    lib.fltee_debug_trace.restype = None
    lib.fltee_debug_trace_text.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    lib.fltee_debug_trace_text.restype = ctypes.c_size_t
    return lib


def traced(fn):
    import torch
    lib = _lib()
    torch.cuda.synchronize()
    lib.fltee_debug_trace(1)
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        lib.fltee_debug_trace(0)
    n = lib.fltee_debug_trace_text(None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.fltee_debug_trace_text(buf, n + 1)
    return buf.value.decode().splitlines()


def assert_same_trace(a, b, what):
    assert a, f"{what}: empty trace"
    if a != b:
        i = next((j for j, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
        raise AssertionError(f"{what}: traces differ at line {i} of {len(a)} / {len(b)}: "
                             f"{a[i] if i < len(a) else None!r} vs {b[i] if i < len(b) else None!r}")


def uploads(rng, n, d, k, kind):
    """client-major (idx, val) with the same sizes: random distinct indices per client, or
    adversarial (client 0 repeating one index; every record on one index)"""
    idx = np.concatenate([rng.choice(d, k, replace=False) for _ in range(n)]).astype(np.uint32)
    if kind == "one_client":
        idx[:k] = 3
    elif kind == "one_index":
        idx[:] = 3
    elif kind == "dense":
        idx = np.tile(np.arange(d, dtype=np.uint32), n)
    val = rng.normal(0, 0.01, n * k).astype(np.float32)
    return idx, val


KINDS = ("random", "one_client", "one_index")


def _device_traces(dev, alg, n, d, k, kinds, **kw):
    import torch
    recs = []
    for i, kind in enumerate(kinds):
        idx, val = uploads(np.random.default_rng(1000 + i), n, d, k, kind)
        recs.append(torch.from_numpy(dev.pack_records(idx, val)).cuda())
    out = torch.empty(d, dtype=torch.float32, device="cuda")

    def run(rec):
        dev.aggregate(alg, rec, n, k, d, out=out, **kw)
        assert dev.status() == 0

    run(recs[0])  # the shape's scratch
    return [traced(lambda r=r: run(r)) for r in recs]


@pytest.mark.parametrize("n,d,k", [(30, 5000, 500),      # fused fold + compaction
                                   (400, 20000, 1000),   # streaming fold + patch
                                   (100, 50890, 5089)])  # configs[2]
def test_advanced_trace_is_data_independent(dev, n, d, k):
    tr = _device_traces(dev, 1, n, d, k, KINDS)
    for t, kind in zip(tr[1:], KINDS[1:]):
        assert_same_trace(tr[0], t, f"advanced n={n} d={d} k={k} {kind}")


@pytest.mark.parametrize("fused", [True, False])
def test_advanced_trace_fold_paths(dev, fused):
    from fltee import _lib as L
    L.lib().fltee_debug_set_fold_compact(1 if fused else 0)
    try:
        tr = _device_traces(dev, 1, 60, 8000, 800, KINDS)
    finally:
        L.lib().fltee_debug_set_fold_compact(1)
    for t, kind in zip(tr[1:], KINDS[1:]):
        assert_same_trace(tr[0], t, f"advanced fused={fused} {kind}")


def test_alg6_trace_is_data_independent(dev):
    tr = _device_traces(dev, 6, 30, 5000, 500, KINDS, batch=7)
    for t, kind in zip(tr[1:], KINDS[1:]):
        assert_same_trace(tr[0], t, f"alg 6 {kind}")


@pytest.mark.parametrize("alg,tree", [(3, False), (5, False), (5, True)])
def test_flat_sparse_trace_is_data_independent(dev, alg, tree):
    # baseline / path_oram's ordered sweep; path_oram as the tree Path ORAM
    tr = _device_traces(dev, alg, 10, 3000, 300, KINDS, oram_tree=tree)
    for t, kind in zip(tr[1:], KINDS[1:]):
        assert_same_trace(tr[0], t, f"alg {alg} tree={tree} {kind}")


@pytest.mark.parametrize("alg", [3, 5])
def test_flat_dense_sized_trace_is_data_independent(dev, alg):
    # k == d sent sparse (the composite-key network's ordered fold)
    tr = _device_traces(dev, alg, 6, 2000, 2000, KINDS)
    for t, kind in zip(tr[1:], KINDS[1:]):
        assert_same_trace(tr[0], t, f"alg {alg} dense-sized {kind}")


@pytest.mark.parametrize("alg", [3, 4, 5])
def test_dense_trace_is_data_independent(dev, alg):
    import torch
    n, d = 20, 100000
    recs = []
    for i in range(2):
        idx, val = uploads(np.random.default_rng(7 + i), n, d, d, "dense")
        recs.append(torch.from_numpy(dev.pack_records(idx, val)).cuda())
    out = torch.empty(d, dtype=torch.float32, device="cuda")

    def run(rec):
        dev.aggregate(alg, rec, n, d, d, out=out, dense=True)
        assert dev.status() == 0

    run(recs[0])
    a, b = traced(lambda: run(recs[0])), traced(lambda: run(recs[1]))
    assert_same_trace(a, b, f"dense alg {alg}")


def test_nips19_trace_is_data_independent(dev):
    tr = _device_traces(dev, 2, 30, 4000, 400, KINDS, seed=4321)
    for t, kind in zip(tr[1:], KINDS[1:]):
        assert_same_trace(tr[0], t, f"nips19 {kind}")


@pytest.mark.parametrize("alg", [1, 3, 6])
@pytest.mark.parametrize("n,d,k", [(5, 3000, 300),         # staged (one DMA each way)
                                   (500, 50890, 5089)])   # pipelined H2D chunks (> 16 MB)
def test_ecall_trace_is_data_independent(oracle, alg, n, d, k):
    import torch

    from fltee.ecalls import Enclave, set_debug_seed
    torch.cuda.init()
    ids = np.arange(40, 40 + n, dtype=np.uint32)
    encs = []
    for i, kind in enumerate(KINDS):
        idx, val = uploads(np.random.default_rng(50 + i), n, d, k, kind)
        w = oracle.as_weights(idx, val).reshape(n, k)
        encs.append(oracle.encrypt_clients(ids, [w[c].tobytes() for c in range(n)]))
    E = Enclave(0)
    fl = [3000 + 10 * alg + (n > 5)]

    def call(enc):
        fl[0] += 100
        set_debug_seed(99)
        try:
            assert E.ecall_fl_init(fl[0], ids, d, k, 1.12, 1.0, 0.1, 1.0, alg, 0, 0) == (0, 0)
            assert E.ecall_start_round(fl[0], 0, n)[:2] == (0, 0)
            if alg == 6:
                st, rv, _, _ = E.ecall_client_size_optimized_secure_aggregation(
                    fl[0], 0, 7, ids, enc, d, k, alg)
            else:
                st, rv, _, _ = E.ecall_secure_aggregation(fl[0], 0, ids, enc, d, k, alg)
        finally:
            set_debug_seed(0)
        assert (st, rv) == (0, 0)

    try:
        call(encs[0])  # the shape's scratch and pinned staging
        tr = [traced(lambda e=e: call(e)) for e in encs]
    finally:
        E.destroy()
    for t, kind in zip(tr[1:], KINDS[1:]):
        assert_same_trace(tr[0], t, f"ECALL alg {alg} n={n} {kind}")

"""The C-ABI library loads and exports every symbol include/fltee_agg.h declares.

CPU-only: no compute entry point is called (no GPU here), except the host-side
AES block self-test which uses the same tables the device kernel stages in LDS.
"""
import ctypes
import os
import re
import subprocess

import numpy as np

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "fltee_agg.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", text)) -
                  {"defined", "sizeof"})


def test_header_declares_the_four_ecalls():
    names = declared_functions()
    for ecall in ("ecall_fl_init", "ecall_start_round", "ecall_secure_aggregation",
                  "ecall_client_size_optimized_secure_aggregation"):
        assert ecall in names


def test_library_exports_every_declared_symbol():
    from fltee import _lib as L
    lib = L.lib()
    names = declared_functions()
    assert names, "no declarations parsed"
    for name in names:
        assert hasattr(lib, name), f"{name} declared in fltee_agg.h but not exported"
        assert name in L.SIGNATURES, f"{name} has no ctypes signature in fltee/_lib.py"
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (\S+)", out))
    assert set(names) <= exported


def source_hash():
    """sha256 of fl-tee_amd/csrc/* (file-name order) + include/fltee_agg.h, first 16 hex
    digits: what fl-tee_amd/Makefile embeds in fltee_version()."""
    import hashlib
    csrc = os.path.join(ROOT, "fl-tee_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(csrc)):
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    with open(HEADER, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def test_version_string():
    from fltee import _lib as L
    assert b"gfx950" in L.lib().fltee_version()


def test_library_built_from_these_sources():
    """Provenance: the loaded libfltee_agg.so was built from the tree's own sources (a
    product build: no A/B tune flags)."""
    from fltee import _lib as L
    v = L.lib().fltee_version().decode()
    if os.environ.get("FLTEE_LIB"):
        return  # an A/B build loaded on purpose
    assert f"src={source_hash()} " in v + " ", f"stale library: {v} vs sources {source_hash()}"
    assert v.endswith("tune="), v


def test_device_aes_tables_fips197():
    # FIPS-197 Appendix C.1 (AES-128)
    from fltee import _lib as L
    key = (ctypes.c_uint8 * 16)(*range(16))
    pt = (ctypes.c_uint8 * 16)(*bytes.fromhex("00112233445566778899aabbccddeeff"))
    out = (ctypes.c_uint8 * 16)()
    L.lib().fltee_debug_aes_block(key, pt, out)
    assert bytes(out).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_device_aes_tables_match_ctr_keystream(oracle):
    # keystream block b of AES-128-CTR (zero IV) = AES_k(BE128(b))
    from fltee import _lib as L
    key = oracle.session_key(4242)
    ks = oracle.aes128_ctr(key, bytes(48))
    for b in range(3):
        ctr = (ctypes.c_uint8 * 16)(*([0] * 15 + [b]))
        out = (ctypes.c_uint8 * 16)()
        L.lib().fltee_debug_aes_block((ctypes.c_uint8 * 16)(*key.tolist()), ctr, out)
        assert bytes(out) == ks[16 * b:16 * b + 16]


def test_no_cpu_fallback_when_library_missing(tmp_path, monkeypatch):
    from fltee import _lib as L
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(L, "_lib", None)
    try:
        L.lib()
    except RuntimeError as e:
        assert "no CPU fallback" in str(e)
    else:
        raise AssertionError("loading a missing library must fail loudly")


def test_pack_records_roundtrip():
    from fltee.device import pack_records, unpack_records
    idx = np.array([0, 7, 0xFFFFFFFF], np.uint32)
    val = np.array([1.5, -0.0, np.inf], np.float32)
    r = pack_records(idx, val)
    i2, v2 = unpack_records(r)
    assert np.array_equal(i2, idx) and np.array_equal(v2.view(np.uint32), val.view(np.uint32))
    # byte layout == Weight (parameters.rs:9): [u32 LE idx][f32 LE val]
    w = np.frombuffer(r.tobytes(), dtype=[("idx", "<u4"), ("val", "<f4")])
    assert np.array_equal(w["idx"], idx)


def test_session_round_keys_aesni_equals_portable():
    """The ECALL's per-client AES-128 key schedules: the AES-NI path (host_aesni.cpp) and
    the portable bitsliced circuit (k_aes.hip) give the same 44 round-key words, and the
    first four are the session key of session_key_store.rs:17-32 (id big-endian in bytes
    4..8)."""
    from fltee import _lib as L
    lib = L.lib()
    rng = np.random.default_rng(7)
    ids = np.concatenate([[0, 1, 0xFFFF, 0xFFFFFFFF], rng.integers(0, 2 ** 32, 60)]).astype(np.uint32)
    n = len(ids)
    a = np.zeros(n * 44, np.uint32)
    b = np.zeros(n * 44, np.uint32)
    used = lib.fltee_debug_session_round_keys(ids.ctypes.data, n, a.ctypes.data, 0)
    lib.fltee_debug_session_round_keys(ids.ctypes.data, n, b.ctypes.data, 1)
    assert np.array_equal(a, b), f"AES-NI path used: {used}"
    w = a.reshape(n, 44)
    assert (w[:, 0] == 0).all() and (w[:, 2] == 0).all() and (w[:, 3] == 0).all()
    assert np.array_equal(w[:, 1], ids)


RAW_GPU_CALLS = ("hipLaunchKernelGGL", "hipMemcpyAsync", "hipMemcpy2DAsync", "hipMemcpy",
                 "hipMemsetAsync", "hipMemset", "hipStreamSynchronize", "hipDeviceSynchronize",
                 "hipEventSynchronize")


def test_every_launch_copy_and_sync_goes_through_the_trace():
    """the obliviousness test (tests/test_gpu_oblivious.py) compares launch
    traces; a launch, copy, memset or host synchronisation that bypassed the trace
    wrappers of csrc/common.h (FLTEE_LAUNCH, fl_memcpy_async, fl_memset_async,
    fl_stream_sync, ...) would be invisible to it.  Every .hip source is scanned (comments
    stripped); the raw calls may appear only inside those wrappers in common.h."""
    csrc = os.path.join(ROOT, "fl-tee_amd", "csrc")
    pat = re.compile(r"(?<![A-Za-z0-9_])(" + "|".join(RAW_GPU_CALLS) + r")\s*\(")
    bad = []
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".hip", ".cpp")):
            continue
        text = open(os.path.join(csrc, f)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for i, line in enumerate(text.splitlines(), 1):
            code = line.split("//", 1)[0]
            for m in pat.finditer(code):
                bad.append(f"{f}:{i}: {m.group(1)}")
    assert not bad, "raw GPU calls outside the trace wrappers:\n" + "\n".join(bad)
    common = open(os.path.join(csrc, "common.h")).read()
    for w in ("FLTEE_LAUNCH", "fl_memcpy_async", "fl_memset_async", "fl_stream_sync", "fl_device_sync"):
        assert w in common
    # and the library exports the trace hooks the GPU test drives
    from fltee import _lib as L
    for sym in ("fltee_debug_trace", "fltee_debug_trace_text"):
        assert hasattr(L.lib(), sym)

"""The compiled C host (tests/abi_host.c) over include/fltee_agg.h.

abi_host.c re-declares the four ECALLs exactly as the Rust FFI block does
(secure_aggregation/app/src/ecalls.rs:6-64) and runs server.rs:44-215's call
sequence (fl_init -> start_round(0) -> aggregate -> start_round(1)).  The CPU
tests prove the declaration check bites and that the binary links; the GPU tests
run it on the reference client's payloads and compare with the oracle's restated
enclave and with the reference's own aggregate (tests/refcheck.py).
"""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import refcheck as R
from conftest import ROOT, gpu_available

BIN = os.path.join(ROOT, "tests", "abi_host")
SRC = os.path.join(ROOT, "tests", "abi_host.c")
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "fl-tee_amd", "lib")


def _compile(src_text, out):
    with tempfile.NamedTemporaryFile("w", suffix=".c", delete=False) as f:
        f.write(src_text)
        path = f.name
    try:
        return subprocess.run(["gcc", "-std=gnu11", "-O0", "-Wall", "-Werror", "-I", INC, path,
                               "-L", LIBDIR, "-lfltee_agg", "-o", out],
                              capture_output=True, text=True)
    finally:
        os.unlink(path)


@pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libfltee_agg.so")),
                    reason="library not built")
def test_abi_host_compiles_against_header(tmp_path):
    r = _compile(open(SRC).read(), str(tmp_path / "h"))
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libfltee_agg.so")),
                    reason="library not built")
@pytest.mark.parametrize("bad", [
    # client_size as u32 instead of usize
    ("const uint32_t *client_ids, size_t client_size,\n                                  size_t num_of_parameters",
     "const uint32_t *client_ids, uint32_t client_size,\n                                  size_t num_of_parameters"),
    # execution_time_results as f64
    ("float *updated_parameters_data,\n                                             float *execution_time_results);",
     "float *updated_parameters_data,\n                                             double *execution_time_results);"),
])
def test_abi_drift_is_a_build_error(tmp_path, bad):
    """The check is real: a prototype that drifts from ecalls.rs does not compile."""
    text = open(SRC).read()
    assert bad[0] in text
    r = _compile(text.replace(bad[0], bad[1]), str(tmp_path / "h"))
    assert r.returncode != 0 and "conflicting types" in r.stderr


def write_input(path, ids, slices, alg, d, k, optimal, fl_id=7, ratio=1.0, dp=0):
    bpc = len(slices[0])
    with open(path, "wb") as f:
        f.write(struct.pack("<IIIIQQQfIQ", 0x48544C46, len(ids), alg, fl_id, d, k, optimal, ratio,
                            dp, bpc))
        f.write(np.asarray(ids, np.uint32).tobytes())
        for s in slices:
            assert len(s) == bpc
            f.write(s)


def read_output(path, n, d):
    b = open(path, "rb").read()
    o = 0
    rvs = np.frombuffer(b, np.uint32, 4, o); o += 16
    sampled = np.frombuffer(b, np.uint32, n, o); o += 4 * n
    upd = np.frombuffer(b, np.float32, d, o); o += 4 * d
    times = np.frombuffer(b, np.float32, 4, o); o += 16
    nxt = struct.unpack_from("<I", b, o)[0]; o += 4
    next_ids = np.frombuffer(b, np.uint32, n, o); o += 4 * n
    assert o == len(b)
    return rvs, sampled, upd, times, nxt, next_ids


@pytest.mark.skipif(gpu_available() or not os.path.exists(BIN), reason="CPU-only check")
def test_abi_host_runs_and_reports_no_device(oracle, tmp_path):
    c = R.case("dense_n4")
    w = R.records(c).reshape(c["n"], c["k"])
    slices = [oracle.aes128_ctr(oracle.session_key(i), w[j].tobytes())
              for j, i in enumerate(c["client_ids"])]
    write_input(tmp_path / "in", c["client_ids"], slices, 4, c["d"], c["k"], 1)
    r = subprocess.run([BIN, str(tmp_path / "in"), str(tmp_path / "out")], capture_output=True, text=True)
    assert r.returncode == 3, (r.returncode, r.stderr)


CASES = [("sparse_n32", 4, 1), ("sparse_n32", 1, 1), ("sparse_n30", 3, 1), ("dense_n30", 5, 1),
         ("sparse_n4", 6, 2), ("sparse_n30", 2, 1)]


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("name,alg,optimal", CASES)
def test_abi_host_server_sequence(oracle, tmp_path, name, alg, optimal):
    c = R.case(name)
    n, d, k = c["n"], c["d"], c["k"]
    ids = c["client_ids"]
    w = R.records(c).reshape(n, k)
    slices = [oracle.aes128_ctr(oracle.session_key(int(i)), w[j].tobytes()) for j, i in enumerate(ids)]
    write_input(tmp_path / "in", ids, slices, alg, d, k, optimal)
    r = subprocess.run([BIN, str(tmp_path / "in"), str(tmp_path / "out")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    rvs, sampled, upd, times, nxt, next_ids = read_output(tmp_path / "out", n, d)
    assert (rvs == 0).all() and nxt == 1
    assert np.array_equal(sampled, ids) and np.array_equal(next_ids, ids)  # ratio 1.0: all, in order
    assert np.isfinite(times).all() and (times >= 0).all()
    enc = b"".join(slices)
    if alg == 2:  # random Laplace counts / shuffle key: the reference criterion only
        R.assert_reassociated(upd, c)
        return
    O = oracle.OracleEnclave(seed=3)
    assert O.fl_init(9, ids, d, k, 1.12, 1.0, 0.1, 1.0, alg) == 0
    assert O.start_round(9, 0, n)[0] == 0
    if alg == 6:
        st, ref, _ = O.client_size_optimized_secure_aggregation(9, 0, optimal, ids, enc, d, k, alg)
    else:
        st, ref, _ = O.secure_aggregation(9, 0, ids, enc, d, k, alg)
    assert st == 0 and np.array_equal(upd.view(np.uint32), ref.view(np.uint32))
    if alg in (3, 4, 5):
        R.assert_in_order_exact(upd, c)
    else:
        R.assert_reassociated(upd, c)

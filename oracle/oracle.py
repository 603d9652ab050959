"""ctypes wrapper over liboracle.so — the CPU restatement of FL-TEE's enclave.

TEST INFRASTRUCTURE ONLY.  Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, and only as the checker / the timed CPU
baseline; the product (fl-tee_amd/) never imports it.  Parity status of each
function is stated in oracle/fltee_oracle.h.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_AES_PATH = os.path.join(HERE, "_ref", "libsgx_enc.so")

WEIGHT = np.dtype([("idx", "<u4"), ("val", "<f4")])  # parameters.rs:9

SUCCESS, UNEXPECTED, INVALID_PARAMETER, ENCLAVE_CRASHED = 0x0, 0x1, 0x2, 0x1006

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, S, U32, U64, F, U8 = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                 ctypes.c_uint64, ctypes.c_float, ctypes.c_uint8)
        sig = {
            "fo_philox4x32_10": (None, [P, P, P]),
            "fo_mix32": (U32, [U32]),
            "fo_shuffle_step_key": (U32, [U32, U32, U32]),
            "fo_session_key": (None, [U32, P]),
            "fo_aes128_ctr": (ctypes.c_int, [P, P, S, P]),
            "fo_decrypt_and_parse": (ctypes.c_int, [P, S, P, S, P, P]),
            "fo_average_params": (None, [P, S, S]),
            "fo_non_oblivious": (U32, [P, S, P, S, S]),
            "fo_baseline": (None, [P, S, P, S, S]),
            "fo_path_oram": (U32, [P, S, P, S, S]),
            "fo_bitonic_sort_by_idx": (None, [P, S]),
            "fo_fold": (None, [P, S]),
            "fo_next_pow2": (S, [S]),
            "fo_advanced_core": (U32, [S, S, P, S, S, P, S]),
            "fo_advanced": (U32, [S, P, S, P, S, S, P, S]),
            "fo_client_size_optimized": (U32, [S, S, P, S, P, S, P, S]),
            "fo_nips19_threshold": (F, [S, S, S]),
            "fo_laplace_r": (None, [S, S, S, U64, P, P]),
            "fo_oblivious_pad": (S, [P, S, F, P]),
            "fo_shuffle_keyed": (None, [P, S, U32]),
            "fo_shuffle_fxhash": (None, [P, S]),
            "fo_safe_aggregate": (None, [P, S, P, S, S]),
            "fo_nips19": (U32, [S, P, S, P, S, S, U64, ctypes.c_int, P, S]),
            "fo_dp_noise": (None, [P, S, F, F, S, U64]),
            "fo_l2_clip": (None, [P, S, F]),
            "fo_sample_client_ids": (None, [P, S, S, U64, P]),
            "fo_reset": (None, []),
            "fo_set_seed": (None, [U64]),
            "fo_set_threads": (None, [ctypes.c_int]),
            "fo_ecall_fl_init": (U32, [U32, P, S, S, S, F, F, F, F, U32, U8, U8]),
            "fo_ecall_start_round": (U32, [U32, U32, S, P]),
            "fo_ecall_secure_aggregation": (U32, [U32, U32, P, S, P, S, S, S, U32, P, P]),
            "fo_ecall_client_size_optimized_secure_aggregation":
                (U32, [U32, U32, S, P, S, P, S, S, U32, P, P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def as_weights(idx, val):
    w = np.empty(len(idx), dtype=WEIGHT)
    w["idx"] = idx
    w["val"] = val
    return w


# ---------------------------------------------------------------- RNG ------
def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib().fo_philox4x32_10(_p(c), _p(k), _p(o))
    return o


# ------------------------------------------------------------- crypto ------
def session_key(client_id):
    k = np.zeros(16, dtype=np.uint8)
    lib().fo_session_key(client_id, _p(k))
    return k


def aes128_ctr(key, data):
    src = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    dst = np.zeros_like(src)
    k = np.frombuffer(bytes(key), dtype=np.uint8).copy() if isinstance(key, (bytes, bytearray)) \
        else np.asarray(key, dtype=np.uint8)
    assert lib().fo_aes128_ctr(_p(k), _p(src), len(src), _p(dst)) == 0
    return dst.tobytes()


def encrypt_clients(client_ids, payloads):
    """Client side of the wire (utils.py:268-304): AES-CTR per client, concatenated."""
    return b"".join(aes128_ctr(session_key(c), p) for c, p in zip(client_ids, payloads))


def decrypt_and_parse(client_ids, enc):
    ids = np.asarray(client_ids, dtype=np.uint32)
    src = np.frombuffer(bytes(enc), dtype=np.uint8).copy()
    n = len(ids)
    out = np.zeros(len(src) // 8 + 1, dtype=WEIGHT)
    nout = ctypes.c_size_t(0)
    assert lib().fo_decrypt_and_parse(_p(ids), n, _p(src), len(src), _p(out),
                                      ctypes.byref(nout)) == 0
    return out[: nout.value]


# ------------------------------------------------------- aggregations ------
def _w(w):
    return np.ascontiguousarray(w, dtype=WEIGHT)


def non_oblivious(w, d, n):
    w = _w(w)
    g = np.zeros(d, dtype=np.float32)
    st = lib().fo_non_oblivious(_p(g), d, _p(w), len(w), n)
    return g, st


def baseline(w, d, n):
    w = _w(w)
    g = np.zeros(d, dtype=np.float32)
    lib().fo_baseline(_p(g), d, _p(w), len(w), n)
    return g


def path_oram(w, d, n):
    w = _w(w)
    g = np.zeros(d, dtype=np.float32)
    st = lib().fo_path_oram(_p(g), d, _p(w), len(w), n)
    return g, st


def bitonic_sort(s):
    s = _w(s).copy()
    assert len(s) & (len(s) - 1) == 0
    lib().fo_bitonic_sort_by_idx(_p(s), len(s))
    return s


def fold(s, fold_len):
    s = _w(s).copy()
    lib().fo_fold(_p(s), fold_len)
    return s


def next_pow2(x):
    return lib().fo_next_pow2(x)


def advanced_core(k_req, d, w, n):
    """_advanced (advanced.rs:39-113): returns the post-sort-2 array (len = nw + d)."""
    w = _w(w)
    cap = next_pow2(len(w) + d)
    scratch = np.zeros(cap, dtype=WEIGHT)
    st = lib().fo_advanced_core(k_req, d, _p(w), len(w), n, _p(scratch), cap)
    return scratch[: len(w) + d], st


def advanced(k_req, w, d, n):
    w = _w(w)
    cap = next_pow2(len(w) + d)
    scratch = np.zeros(cap, dtype=WEIGHT)
    g = np.zeros(d, dtype=np.float32)
    st = lib().fo_advanced(k_req, _p(g), d, _p(w), len(w), n, _p(scratch), cap)
    return g, st


def client_size_optimized(batch, k, w, d, n):
    w = _w(w)
    cap = next_pow2(min(batch, n) * k + d)
    scratch = np.zeros(cap, dtype=WEIGHT)
    g = np.zeros(d, dtype=np.float32)
    st = lib().fo_client_size_optimized(batch, k, _p(g), d, _p(w), n, _p(scratch), cap)
    return g, st


def nips19_threshold(d, k, n):
    return lib().fo_nips19_threshold(d, k, n)


def laplace_r(d, k, n, seed):
    r = np.zeros(d, dtype=np.uint32)
    T = ctypes.c_float(0)
    lib().fo_laplace_r(d, k, n, seed, _p(r), ctypes.byref(T))
    return r, T.value


def oblivious_pad(r, d, T):
    r = np.ascontiguousarray(r, dtype=np.uint32)
    out = np.zeros(d * int(T) if T > 0 else 0, dtype=WEIGHT)
    m = lib().fo_oblivious_pad(_p(r), d, T, _p(out))
    return out[:m]


def shuffle_keyed(s, seed):
    s = _w(s).copy()
    lib().fo_shuffle_keyed(_p(s), len(s), seed)
    return s


def shuffle_fxhash(s):
    s = _w(s).copy()
    lib().fo_shuffle_fxhash(_p(s), len(s))
    return s


def safe_aggregate(s, d, n):
    s = _w(s)
    g = np.zeros(d, dtype=np.float32)
    lib().fo_safe_aggregate(_p(g), d, _p(s), len(s), n)
    return g


def nips19(k, w, d, n, seed, reference_shuffle=False):
    w = _w(w)
    T = nips19_threshold(d, k, n)
    cap = next_pow2(len(w) + d * max(int(T), 0))
    scratch = np.zeros(cap, dtype=WEIGHT)
    g = np.zeros(d, dtype=np.float32)
    st = lib().fo_nips19(k, _p(g), d, _p(w), len(w), n, seed, int(reference_shuffle),
                         _p(scratch), cap)
    return g, st


def dp_noise(g, sigma, clipping, n, seed):
    g = np.ascontiguousarray(g, dtype=np.float32).copy()
    lib().fo_dp_noise(_p(g), len(g), sigma, clipping, n, seed)
    return g


def l2_clip(vals, clipping):
    v = np.ascontiguousarray(vals, dtype=np.float32).copy()
    lib().fo_l2_clip(_p(v), len(v), clipping)
    return v


def sample_client_ids(ids, amount, seed):
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    out = np.zeros(amount, dtype=np.uint32)
    lib().fo_sample_client_ids(_p(ids), len(ids), amount, seed, _p(out))
    return out


def set_threads(t):
    """Tests only: run the comparator networks on t threads (results are identical)."""
    lib().fo_set_threads(int(t))


# ------------------------------------------------------ ECALL mirror ------
class OracleEnclave:
    """The lib.rs ECALL state machine, restated (process-global like the enclave)."""

    def __init__(self, seed=None):
        lib().fo_reset()
        if seed is not None:
            lib().fo_set_seed(seed)

    def fl_init(self, fl_id, client_ids, d, k, sigma, clipping, alpha, ratio, alg,
                verbose=0, dp=0):
        ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
        return lib().fo_ecall_fl_init(fl_id, _p(ids), len(ids), d, k, sigma, clipping, alpha,
                                      ratio, alg, verbose, dp)

    def start_round(self, fl_id, rnd, sample_size):
        out = np.zeros(max(sample_size, 1), dtype=np.uint32)
        st = lib().fo_ecall_start_round(fl_id, rnd, sample_size, _p(out))
        return st, out[:sample_size]

    def secure_aggregation(self, fl_id, rnd, client_ids, enc, d, k, alg):
        ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
        src = np.frombuffer(bytes(enc), dtype=np.uint8).copy()
        out = np.full(d, np.nan, dtype=np.float32)
        times = np.zeros(3, dtype=np.float32)
        st = lib().fo_ecall_secure_aggregation(fl_id, rnd, _p(ids), len(ids), _p(src), len(src),
                                               d, k, alg, _p(out), _p(times))
        return st, out, times

    def client_size_optimized_secure_aggregation(self, fl_id, rnd, batch, client_ids, enc, d,
                                                 k, alg):
        ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
        src = np.frombuffer(bytes(enc), dtype=np.uint8).copy()
        out = np.full(d, np.nan, dtype=np.float32)
        times = np.zeros(3, dtype=np.float32)
        st = lib().fo_ecall_client_size_optimized_secure_aggregation(
            fl_id, rnd, batch, _p(ids), len(ids), _p(src), d, k, alg, _p(out), _p(times))
        return st, out, times


# ------------------------------------------------ reference AES library ----
def ref_aes_available():
    return os.path.exists(REF_AES_PATH)


def ref_aes_ctr_encrypt(key, data):
    """The reference's own sgx_aes_ctr_encrypt (src/cpp/encryption.cpp) built into _ref/."""
    L = ctypes.CDLL(REF_AES_PATH)
    src = (ctypes.c_uint8 * len(data)).from_buffer_copy(bytes(data))
    dst = (ctypes.c_uint8 * len(data))()
    k = (ctypes.c_uint8 * 16)(*list(key))
    ctr = (ctypes.c_uint8 * 16)()
    rc = L.sgx_aes_ctr_encrypt(k, src, ctypes.c_uint32(len(data)), ctr, ctypes.c_uint32(128), dst)
    assert rc == 0
    return bytes(dst)

"""Host-side mirror of secure_aggregation/app/src/ecalls.rs over the C ABI.

`Enclave` replaces `init_enclave()` / `SgxEnclave` (ecalls.rs:66-83) and
exposes the four ECALLs with the argument meaning of ecalls.rs:6-64.  Each
method returns `(bridge_status, retval, ...)` exactly like the Rust host sees
them (`result`, `retval`): the server panics unless both are SUCCESS
(server.rs:80-82,96-98,159-161,180-182,202-204).
"""
import ctypes

import numpy as np

from . import _lib as L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _as_u8(buf):
    """bytes / bytearray / numpy array -> flat uint8 view (no copy of large payloads)."""
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    if isinstance(buf, (bytes, bytearray, memoryview)):
        return np.frombuffer(buf, dtype=np.uint8)
    return np.frombuffer(bytes(buf), dtype=np.uint8)  # e.g. fl_main.py's list of ints


class Enclave:
    """device: one HIP device id, or a list of them for an eid over several GPUs
    (fltee_device_init_multi: the ECALLs shard internally; the same id repeated gives
    virtual ranks on one GPU)."""

    def __init__(self, device=0):
        self.lib = L.lib()
        eid = ctypes.c_uint64(0)
        if isinstance(device, (list, tuple)):
            devs = (ctypes.c_int * len(device))(*device)
            st = self.lib.fltee_device_init_multi(devs, len(device), ctypes.byref(eid))
        else:
            st = self.lib.fltee_device_init(device, ctypes.byref(eid))
        if st != L.SUCCESS:
            raise RuntimeError(f"fltee_device_init({device}) failed: {st:#x}")
        self.eid = eid.value

    def device_count(self):
        return self.lib.fltee_device_count(self.eid)

    def geteid(self):
        return self.eid

    def destroy(self):
        if self.eid:
            self.lib.fltee_device_fini(self.eid)
            self.eid = 0

    # lib.rs:113-180
    def ecall_fl_init(self, fl_id, client_ids, num_of_parameters, num_of_sparse_parameters,
                      sigma, clipping, alpha, sampling_ratio, aggregation_alg, verbose, dp):
        ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
        rv = ctypes.c_uint32(0xFFFFFFFF)
        st = self.lib.ecall_fl_init(self.eid, ctypes.byref(rv), fl_id, _p(ids), len(ids),
                                    num_of_parameters, num_of_sparse_parameters, sigma, clipping,
                                    alpha, sampling_ratio, aggregation_alg, int(verbose), int(dp))
        return st, rv.value

    # lib.rs:182-219
    def ecall_start_round(self, fl_id, round_, sample_size):
        out = np.zeros(max(sample_size, 1), dtype=np.uint32)
        rv = ctypes.c_uint32(0xFFFFFFFF)
        st = self.lib.ecall_start_round(self.eid, ctypes.byref(rv), fl_id, round_, sample_size,
                                        _p(out))
        return st, rv.value, out[:sample_size]

    # lib.rs:221-423
    def ecall_secure_aggregation(self, fl_id, round_, client_ids, encrypted_parameters,
                                 num_of_parameters, num_of_sparse_parameters, aggregation_alg):
        ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
        enc = _as_u8(encrypted_parameters)
        out = np.empty(num_of_parameters, dtype=np.float32)  # written whole by the call
        times = np.full(3, np.nan, dtype=np.float32)
        rv = ctypes.c_uint32(0xFFFFFFFF)
        st = self.lib.ecall_secure_aggregation(
            self.eid, ctypes.byref(rv), fl_id, round_, _p(ids), len(ids), _p(enc), enc.nbytes,
            num_of_parameters, num_of_sparse_parameters, aggregation_alg, _p(out), _p(times))
        return st, rv.value, out, times

    # lib.rs:425-592
    def ecall_client_size_optimized_secure_aggregation(self, fl_id, round_, optimal_num_of_clients,
                                                       client_ids, encrypted_parameters,
                                                       num_of_parameters, num_of_sparse_parameters,
                                                       aggregation_alg):
        ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
        enc = _as_u8(encrypted_parameters)
        need = len(ids) * num_of_sparse_parameters * 8
        if enc.nbytes < need:  # [user_check]: the enclave would read past the buffer
            raise ValueError(f"payload has {enc.nbytes} bytes, alg 6 reads {need}")
        out = np.full(num_of_parameters, np.nan, dtype=np.float32)
        times = np.full(3, np.nan, dtype=np.float32)
        rv = ctypes.c_uint32(0xFFFFFFFF)
        st = self.lib.ecall_client_size_optimized_secure_aggregation(
            self.eid, ctypes.byref(rv), fl_id, round_, optimal_num_of_clients, _p(ids), len(ids),
            _p(enc), num_of_parameters, num_of_sparse_parameters, aggregation_alg, _p(out),
            _p(times))
        return st, rv.value, out, times


def set_debug_seed(seed):
    """Deterministic RNG for sampling / nips19 / DP (tests only; 0 restores RDRAND-like)."""
    L.lib().fltee_debug_set_seed(seed)


def set_path_oram_tree(on):
    """aggregation_alg 5 through the ECALLs: the tree Path ORAM (oram.rs:64-118) when on, the
    output-equivalent oblivious sweep (default) when off (fltee_set_path_oram_tree)."""
    L.lib().fltee_set_path_oram_tree(1 if on else 0)


def set_advanced_exact_runs(on):
    """aggregation_alg 1 and 6 through the ECALLs when some index has a run of more than
    n + 1 entries (a client repeated an index): off (default) answers at the fixed cost of
    the halo fold plus its long-run carry (that run's sum re-associated at the walk
    boundaries); on folds any run exactly, as advanced.rs:66-101 does, at the public
    worst-case cost (fltee_set_advanced_exact_runs)."""
    L.lib().fltee_set_advanced_exact_runs(1 if on else 0)

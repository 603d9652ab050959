"""fltee — MI355X-native drop-in for FL-TEE's SGX aggregation enclave.

The product is the HIP library fl-tee_amd/lib/libfltee_agg.so behind the C ABI
in include/fltee_agg.h.  This package is the host-side mirror of the
reference's interface for that path:

  fltee.ecalls   — ecalls.rs:6-83 (Enclave = init_enclave + the four ECALLs)
  fltee.server   — the Aggregator service logic of app/src/server.rs:44-215
  fltee.device   — device-resident aggregation on torch tensors (bench, tests)
  fltee.parallel — one process per GPU: parameter-range / client-range shards,
                   final RCCL collective over xGMI
"""
from . import _lib
from ._lib import ALG_CODES, LIB_PATH, lib  # noqa: F401

__all__ = ["ALG_CODES", "LIB_PATH", "lib"]

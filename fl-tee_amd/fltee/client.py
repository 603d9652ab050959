"""Client-side producers on the GPU, named after the reference's
client functions in src/utils.py / src/update.py.

fl_main.py:221-238 turns each sampled client's update into its upload:

    top, idxs = zero_except_top_k_weights(diff, buffer_names, k)   # utils.py:327-354
    if dp: top = l2clipping(top, buffer_names, clipping)            # update.py:187-204
    b = serialize_sparse(top, buffer_names, idxs)                   # utils.py:193-209
    (dense: l2clipping + serialize_dense, utils.py:171-190)
    enc = encrypt_parameters(b, client_id)                          # utils.py:268-290

and concatenates the clients' ciphertexts in sampling order.  Here the n clients'
flattened learnable parameters are one [n, d] f32 CUDA tensor and every step is a
kernel of libfltee_agg (no CPU path):

    payload = produce_payloads(values, client_ids, k=k, clipping=C)   # uint8 CUDA tensor

The payload can go into an Aggregate request as is, or straight to the device-side
aggregation (fltee_decrypt_device + fltee_aggregate_device) for a GPU-resident round.
"""
import ctypes

import numpy as np
import torch

from . import _lib as L
from .device import _check, _ptr, _stream


def _values(values):
    assert values.is_cuda and values.dtype == torch.float32 and values.dim() == 2
    return values.contiguous()


def zero_except_top_k_weights(values, k, stream=None):
    """[n, d] -> int64 records [n*k]: (idx, val) of the k largest |val| per client in the
    reference's order (|val| descending, ties by ascending idx)."""
    v = _values(values)
    n, d = v.shape
    rec = torch.empty(n * k, dtype=torch.int64, device=v.device)
    _check(L.lib().fltee_client_topk_device(_ptr(v), n, d, k, _ptr(rec), _stream(stream)),
           "fltee_client_topk_device")
    return rec


def serialize_dense(values, stream=None):
    """[n, d] -> int64 records [n*d]: (i, v[i])."""
    v = _values(values)
    n, d = v.shape
    rec = torch.empty(n * d, dtype=torch.int64, device=v.device)
    _check(L.lib().fltee_client_serialize_dense_device(_ptr(v), n, d, _ptr(rec), _stream(stream)),
           "fltee_client_serialize_dense_device")
    return rec


def l2clipping(records, n, k, clipping, stream=None):
    """In place on n clients x k records: val *= min(1, clipping / ||values||_2)."""
    assert records.is_cuda and records.dtype == torch.int64 and records.numel() >= n * k
    _check(L.lib().fltee_client_clip_device(_ptr(records), n, k, float(clipping), _stream(stream)),
           "fltee_client_clip_device")
    return records


def encrypt_parameters(records, client_ids, stream=None):
    """Records of n clients (equal counts) -> uint8 ciphertext, client-major."""
    ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
    n = len(ids)
    plain = records.contiguous().view(torch.uint8)
    assert plain.numel() % n == 0
    out = torch.empty_like(plain)
    _check(L.lib().fltee_encrypt_device(ids.ctypes.data_as(ctypes.c_void_p), n, _ptr(plain),
                                        plain.numel() // n, _ptr(out), _stream(stream)),
           "fltee_encrypt_device")
    return out


def produce_payloads(values, client_ids, k=None, clipping=None, stream=None):
    """fl_main.py:221-238 for every client at once: k=None -> dense uploads."""
    v = _values(values)
    n, d = v.shape
    assert len(client_ids) == n
    if k is None:
        rec, kk = serialize_dense(v, stream), d
    else:
        rec, kk = zero_except_top_k_weights(v, k, stream), k
    if clipping is not None:
        l2clipping(rec, n, kk, clipping, stream)
    return encrypt_parameters(rec, client_ids, stream)

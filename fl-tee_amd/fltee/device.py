"""Device-resident entry points of libfltee_agg.so on torch tensors.

PyTorch only supplies HBM allocations, the stream and torch.distributed; all
arithmetic runs in the library's HIP kernels.  Records are int64 tensors whose
bytes are the enclave's Weight layout (parameters.rs:9): low 32 bits u32 idx,
high 32 bits f32 val (little-endian), client-major in upload order.
"""
import ctypes

import numpy as np
import torch

from . import _lib as L


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def pack_records(idx, val):
    """(u32 idx, f32 val) arrays -> int64 numpy array of Weight records."""
    idx = np.ascontiguousarray(idx, dtype=np.uint32)
    val = np.ascontiguousarray(val, dtype=np.float32)
    rec = np.empty(len(idx), dtype=np.uint64)
    rec[:] = idx.astype(np.uint64) | (val.view(np.uint32).astype(np.uint64) << np.uint64(32))
    return rec.view(np.int64)


def unpack_records(rec):
    r = np.ascontiguousarray(rec).view(np.uint64)
    return (r & np.uint64(0xFFFFFFFF)).astype(np.uint32), (r >> np.uint64(32)).astype(np.uint32).view(np.float32)


def opts(*, dense=False, dp=False, clip=False, accumulate=False, no_average=False, sigma=1.12,
         clipping=1.0, seed=0, k_req=None, batch=0, n_avg=0, fold_halo=0, status=None,
         oram_tree=False, oram_lazy=False):
    o = L.DeviceOpts()
    o.flags = ((L.OPT_DENSE if dense else 0) | (L.OPT_DP if dp else 0) | (L.OPT_CLIP if clip else 0)
               | (L.OPT_ACCUMULATE if accumulate else 0) | (L.OPT_NO_AVERAGE if no_average else 0)
               | (L.OPT_ORAM_TREE if oram_tree else 0) | (L.OPT_ORAM_LAZY if oram_lazy else 0))
    o.sigma, o.clipping, o.seed = sigma, clipping, seed
    if k_req is not None:
        o.flags |= L.OPT_K_REQ
        o.k_req = k_req
    o.batch, o.n_avg, o.fold_halo = batch, n_avg, fold_halo
    o.d_status = status.data_ptr() if status is not None else None
    return o


def _check(st, what):
    if st != L.SUCCESS:
        raise RuntimeError(f"{what} failed with status {st:#x}")


def aggregate(alg, records, n, k, d, out=None, stream=None, **kw):
    """fltee_aggregate_device: aggregate n x k records (int64 cuda tensor) into out[d] (f32)."""
    assert records.is_cuda and records.dtype == torch.int64 and records.numel() >= n * k
    if out is None:
        out = torch.empty(d, dtype=torch.float32, device=records.device)
    o = opts(**kw)
    st = L.lib().fltee_aggregate_device(alg, _ptr(records), n, k, d, _ptr(out), ctypes.byref(o),
                                        _stream(stream))
    _check(st, "fltee_aggregate_device")
    return out


def reserve(alg, n, k, d, **kw):
    o = opts(**kw)
    _check(L.lib().fltee_reserve(alg, n, k, d, ctypes.byref(o)), "fltee_reserve")


def workspace_bytes(alg, n, k, d, **kw):
    o = opts(**kw)
    return L.lib().fltee_workspace_bytes(alg, n, k, d, ctypes.byref(o))


def status(stream=None):
    """Synchronise and return (and clear) the library-owned device status word."""
    v = ctypes.c_uint32(0)
    _check(L.lib().fltee_device_status(_stream(stream), ctypes.byref(v)), "fltee_device_status")
    return v.value


def bitonic(records, mode, seed=0, stream=None):
    m = records.numel()
    _check(L.lib().fltee_bitonic_device(_ptr(records), m, mode, seed, _stream(stream)),
           "fltee_bitonic_device")
    return records


def fold(src, dst, fold_len, halo, status_word, stream=None):
    _check(L.lib().fltee_fold_device(_ptr(src), _ptr(dst), src.numel(), fold_len, halo,
                                     _ptr(status_word), _stream(stream)), "fltee_fold_device")
    return dst


def decrypt(client_ids, cipher, bytes_per_client, records, stream=None):
    ids = np.ascontiguousarray(client_ids, dtype=np.uint32)
    _check(L.lib().fltee_decrypt_device(ids.ctypes.data_as(ctypes.c_void_p), len(ids),
                                        _ptr(cipher), bytes_per_client, _ptr(records),
                                        _stream(stream)), "fltee_decrypt_device")
    return records


def laplace_r(d, k, n, seed, device="cuda", stream=None):
    r = torch.empty(d, dtype=torch.int32, device=device)
    T = ctypes.c_float(0)
    _check(L.lib().fltee_laplace_r_device(d, k, n, seed, _ptr(r), ctypes.byref(T),
                                          _stream(stream)), "fltee_laplace_r_device")
    return r, T.value


def sum_rows(rows, coef=1.0, out=None, stream=None):
    """fltee_sum_rows_device: out = coef * (rows[0] + rows[1] + ...), added in row order."""
    assert rows.is_cuda and rows.dtype == torch.float32 and rows.dim() == 2
    nrows, d = rows.shape
    rows = rows.contiguous()
    if out is None:
        out = torch.empty(d, dtype=torch.float32, device=rows.device)
    _check(L.lib().fltee_sum_rows_device(_ptr(rows), nrows, d, coef, _ptr(out), _stream(stream)),
           "fltee_sum_rows_device")
    return out


def dp_noise(out, sigma, clipping, n, seed=0, stream=None):
    """fltee_dp_noise_device: out += (N(0, clipping*sigma) / n) as f32 (common.rs:56-72)."""
    _check(L.lib().fltee_dp_noise_device(_ptr(out), out.numel(), sigma, clipping, n, seed,
                                         _stream(stream)), "fltee_dp_noise_device")
    return out


# ---- position-range pieces of `advanced` (multi-GPU Option B, fltee/parallel.py) ----
def advanced_init_range(records, nrec, d, pos_base, m, out=None, stream=None):
    """Entries pos_base..pos_base+m-1 of advanced's padded array (advanced.rs:116-142);
    records[x] is the record at position pos_base + x (read where < nrec)."""
    if out is None:
        out = torch.empty(m, dtype=torch.int64, device=records.device)
    _check(L.lib().fltee_advanced_init_range_device(_ptr(records), nrec, d, pos_base, m, _ptr(out),
                                                    _stream(stream)),
           "fltee_advanced_init_range_device")
    return out


def bitonic_range_sort(records, pos_base, mode=0, seed=0, stream=None, valid=None):
    """valid: entries valid.. of this range are identical pads (None: unknown)."""
    if valid is not None:
        _check(L.lib().fltee_bitonic_range_sort_padded_device(_ptr(records), records.numel(),
                                                              pos_base, valid, mode, seed,
                                                              _stream(stream)),
               "fltee_bitonic_range_sort_padded_device")
        return records
    _check(L.lib().fltee_bitonic_range_sort_device(_ptr(records), records.numel(), pos_base, mode,
                                                   seed, _stream(stream)),
           "fltee_bitonic_range_sort_device")
    return records


def bitonic_range_merge(records, pos_base, stage_log, mode=0, seed=0, stream=None):
    _check(L.lib().fltee_bitonic_range_merge_device(_ptr(records), records.numel(), pos_base, mode,
                                                    seed, stage_log, _stream(stream)),
           "fltee_bitonic_range_merge_device")
    return records


def bitonic_range_exchange(mine, theirs, pos_mine, pos_theirs, stage_log, mode=0, seed=0,
                           stream=None):
    assert theirs.numel() == mine.numel()
    _check(L.lib().fltee_bitonic_range_exchange_device(_ptr(mine), _ptr(theirs), mine.numel(),
                                                       pos_mine, pos_theirs, mode, seed, stage_log,
                                                       _stream(stream)),
           "fltee_bitonic_range_exchange_device")
    return mine


def bitonic_range_steps(records, pos_base, stage_log, step_top, step_bot, mode=0, seed=0,
                        stream=None):
    _check(L.lib().fltee_bitonic_range_steps_device(_ptr(records), records.numel(), pos_base, mode,
                                                    seed, stage_log, step_top, step_bot,
                                                    _stream(stream)),
           "fltee_bitonic_range_steps_device")
    return records


def fold_context(halo):
    return L.lib().fltee_fold_context(halo)


def fold_side_bytes(span, halo):
    return L.lib().fltee_fold_side_bytes(span, halo)


def fold_range(src, dst, origin, end, pos_base, fold_len, halo, side, stream=None):
    """fltee_fold_range_device: [0, origin) of src holds >= fold_context(halo) + 1 records
    of context; side: a byte buffer of >= fold_side_bytes(end - origin, halo)."""
    assert side.numel() * side.element_size() >= fold_side_bytes(end - origin, halo)
    _check(L.lib().fltee_fold_range_device(_ptr(src), _ptr(dst), src.numel(), origin, end, pos_base,
                                           fold_len, halo, _ptr(side), _stream(stream)),
           "fltee_fold_range_device")
    return dst


def fold_range_total(side, span, halo, total, stream=None):
    """the range's segmented total (16 bytes into `total`) for the ranges after it"""
    assert total.numel() * total.element_size() >= 16
    _check(L.lib().fltee_fold_range_total_device(_ptr(side), span, halo, _ptr(total), _stream(stream)),
           "fltee_fold_range_total_device")
    return total


def fold_range_patch(dst, origin, end, pos_base, fold_len, halo, side, prev_totals, stream=None):
    """the long-run patch of one range's fold output; prev_totals: the totals of the ranges
    before it, in order (a contiguous tensor of n * 16 bytes, or None)"""
    n_prev = 0 if prev_totals is None else prev_totals.numel() * prev_totals.element_size() // 16
    _check(L.lib().fltee_fold_range_patch_device(_ptr(dst), origin, end, pos_base, fold_len, halo,
                                                 _ptr(side), _ptr(prev_totals) if n_prev else None,
                                                 n_prev, _stream(stream)),
           "fltee_fold_range_patch_device")
    return dst


def compact_range(chunk, d, coef, buf, tmp, out=None, stream=None):
    if out is None:
        out = torch.empty(d, dtype=torch.float32, device=chunk.device)
    c = chunk.numel()
    assert buf.numel() >= d + c and tmp.numel() >= d + c
    _check(L.lib().fltee_compact_range_device(_ptr(chunk), c, d, _ptr(buf), _ptr(tmp), coef,
                                              _ptr(out), _stream(stream)),
           "fltee_compact_range_device")
    return out


def nips19_build_range(records, nrec, r, d, tf, pos_base, m, out=None, stream=None):
    """Entries pos_base..pos_base+m-1 of nips19's padded array (records ++ Laplace dummies
    ++ pads, common.rs:164-197); r = laplace_r(...)[0], tf = int(T)."""
    if out is None:
        out = torch.empty(m, dtype=torch.int64, device=records.device)
    _check(L.lib().fltee_nips19_build_range_device(_ptr(records), nrec, _ptr(r), d, tf, pos_base, m,
                                                   _ptr(out), _stream(stream)),
           "fltee_nips19_build_range_device")
    return out


def safe_aggregate(entries, d, out=None, stream=None):
    """common.rs:25-35 on a range of shuffled entries: un-averaged f32[d] partial sums."""
    if out is None:
        out = torch.empty(d, dtype=torch.float32, device=entries.device)
    _check(L.lib().fltee_safe_aggregate_device(_ptr(entries), entries.numel(), d, _ptr(out),
                                               _stream(stream)),
           "fltee_safe_aggregate_device")
    return out


def select(entries, d, stream=None):
    """The entries of one range with idx < d, in position order (fltee_select_device):
    the piece of nips19's safe_aggregate a range contributes, as an int64 tensor."""
    count = ctypes.c_size_t(0)
    lst = torch.empty(max(1, entries.numel()), dtype=torch.int64, device=entries.device)
    _check(L.lib().fltee_select_device(_ptr(entries), entries.numel(), d, _ptr(lst), lst.numel(),
                                       ctypes.byref(count), _stream(stream)),
           "fltee_select_device")
    return lst[: count.value]


def ordered_list(lst, d, coef, out=None, stream=None):
    """out[i] = coef * (+0 + v1 + v2 ...) over the list's entries with idx i, in list
    order (fltee_ordered_list_device)."""
    if out is None:
        out = torch.empty(d, dtype=torch.float32, device=lst.device)
    _check(L.lib().fltee_ordered_list_device(_ptr(lst), lst.numel(), d, coef, _ptr(out),
                                             _stream(stream)),
           "fltee_ordered_list_device")
    return out

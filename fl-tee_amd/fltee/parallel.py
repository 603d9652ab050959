"""One process per GPU: sharding the aggregation over the GPUs of one node.

SURVEY §8e.  The enclave is single-threaded; scale-out is new here and follows the
two partitionings the path admits:

* Parameter-range sharding (dense baseline / non_oblivious / path_oram): GPU r owns
  parameters [lo_r, hi_r) of EVERY client and runs the same dense kernel on its
  column slice.  There is no exchange during compute; the averaged shards are
  gathered to the root (RCCL over xGMI) to form the response vector.  Exact: every
  output is still summed over the clients in order by one lane.

* Client-range sharding (advanced, Option A = the reference's own alg 6,
  lib.rs:498-573): GPU r runs `advanced` on clients [c_r, c_{r+1}) and produces an
  un-averaged partial sum; the root adds the partials in rank order
  (fltee_sum_rows_device), scales by 1f32/n and adds DP noise.  With equal shards
  this is bit-identical to alg 6 with batch = n / world.

Collectives go through torch.distributed ("nccl" = RCCL on ROCm; "gloo" in the CPU
tests).  The per-rank compute and the root combine are injectable so the CPU tests
can stand the oracle in for the kernels.
"""
import torch
import torch.distributed as dist


def shard_range(total, world, rank):
    """Even contiguous split of [0, total): rank r gets [lo, hi)."""
    return total * rank // world, total * (rank + 1) // world


def split_dense_columns(values, world, rank):
    """Host/device split of dense client rows [n][d] into this rank's column slice, as
    records with rank-local indices (the layout fltee_aggregate_device expects)."""
    n, d = values.shape
    lo, hi = shard_range(d, world, rank)
    v = values[:, lo:hi].contiguous()
    idx = torch.arange(hi - lo, dtype=torch.int64, device=v.device).expand(n, hi - lo)
    rec = (idx | (v.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
    return rec, lo, hi


def gather_shards(local, d_total, world, rank, root=0):
    """Gather the averaged shards of every rank into the full vector on `root`.
    Shards may differ by one element: they are padded to the largest for the
    collective and trimmed afterwards."""
    if world == 1:
        return local
    width = (d_total + world - 1) // world
    buf = torch.zeros(width, dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, parts, dst=root)
    if rank != root:
        return None
    pieces = []
    for r in range(world):
        lo, hi = shard_range(d_total, world, r)
        pieces.append(parts[r][: hi - lo])
    return torch.cat(pieces)


def param_sharded_dense(values_local_records, n, d_local, d_total, world, rank, alg=3,
                        compute=None, root=0):
    """Dense aggregation of this rank's column slice, then gather to the root."""
    if compute is None:
        from . import device as D

        def compute(rec, n_, d_):
            return D.aggregate(alg, rec, n_, d_, d_, dense=True)
    local = compute(values_local_records, n, d_local)
    return gather_shards(local, d_total, world, rank, root)


def client_sharded_advanced(local_records, n_local, k, d, n_total, world, rank, root=0,
                            compute_partial=None, combine=None, dp=None):
    """Option A: per-rank `advanced` partial sums, combined on the root in rank order.

    dp: None or dict(sigma=..., clipping=..., seed=...) applied on the root after
    averaging (lib.rs:586-588)."""
    if compute_partial is None:
        from . import device as D

        def compute_partial(rec, n_, k_, d_):
            return D.aggregate(1, rec, n_, k_, d_, no_average=True)
    if combine is None:
        from . import device as D

        def combine(rows, coef):
            return D.sum_rows(rows, coef)
    partial = compute_partial(local_records, n_local, k, d)
    coef = float(torch.tensor(1.0, dtype=torch.float32) / torch.tensor(float(n_total), dtype=torch.float32))
    if world == 1:
        rows = partial.reshape(1, -1)
    else:
        parts = [torch.empty_like(partial) for _ in range(world)] if rank == root else None
        dist.gather(partial, parts, dst=root)
        if rank != root:
            return None
        rows = torch.stack(parts)
    out = combine(rows, coef)
    if dp is not None:
        from . import device as D
        D.dp_noise(out, dp["sigma"], dp["clipping"], n_total, dp.get("seed", 0))
    return out

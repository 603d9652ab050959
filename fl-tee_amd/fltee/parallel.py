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

* Position-range sharding (advanced, Option B = the north star's "parameter-index
  range" sharding, configs[4]): `advanced`'s padded array of M entries is split into
  `world` contiguous ranges, one per GPU.  The bitonic network runs distributed — the
  steps with j >= M/world are pairwise exchanges of whole ranges with the partner
  GPU r ^ (j / (M/world)) — so after the sort GPU r holds an index range.  The fold
  takes one halo exchange with the neighbours; each GPU compacts its run
  representatives to their indices and ONE RCCL reduce (sum) over xGMI assembles the
  aggregate on the root.  Same network, same fold: bit-identical to single-GPU
  `advanced`, and every transfer has a fixed size (oblivious).

Collectives go through torch.distributed ("nccl" = RCCL on ROCm; "gloo" in the CPU
tests).  The per-rank compute and the root combine are injectable so the CPU tests
can stand the oracle in for the kernels.
"""
import numpy as np
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


# ------------------------------------------------ Option B: position ranges ----
PAD_RECORD = 0xFFFFFFFF  # (u32::MAX, +0.0) as an int64 record (advanced.rs:133-142)


class DeviceRangeOps:
    """The HIP range pieces (include/fltee_agg.h, fltee.device) as the per-range steps
    of index_sharded_advanced; scratch buffers are kept between calls."""

    def __init__(self):
        from . import device as D
        self.D = D
        self._scratch = {}

    def _buf(self, name, n, dtype, device):
        t = self._scratch.get(name)
        if t is None or t.numel() < n or t.device != device:
            t = torch.empty(n, dtype=dtype, device=device)
            self._scratch[name] = t
        return t[:n]

    def pads(self, n, like):
        return torch.full((n,), PAD_RECORD, dtype=torch.int64, device=like.device)

    def fold_context(self, halo):
        return self.D.fold_context(halo)

    def sort(self, x, pos, mode=0, seed=0, valid=None):
        self.D.bitonic_range_sort(x, pos, mode=mode, seed=seed, valid=valid)

    def merge(self, x, pos, stage_log, mode=0, seed=0):
        self.D.bitonic_range_merge(x, pos, stage_log, mode=mode, seed=seed)

    def exchange(self, x, theirs, pos, pos_theirs, stage_log, mode=0, seed=0):
        self.D.bitonic_range_exchange(x, theirs, pos, pos_theirs, stage_log, mode=mode, seed=seed)

    def safe_aggregate(self, x, d):
        return self.D.safe_aggregate(x, d)

    def select(self, x, d):
        return self.D.select(x, d)

    def ordered(self, lst, d, coef):
        return self.D.ordered_list(lst, d, coef)

    def steps(self, x, pos, stage_log, step_top, step_bot):
        self.D.bitonic_range_steps(x, pos, stage_log, step_top, step_bot)

    def fold(self, buf, origin, end, pos_base, fold_len, halo, key=0):
        """The range's fold into a buffer like `buf` (positions [origin, end) written) and
        its side records (fltee_fold_range_device)."""
        dst = self._buf(("fold", key), buf.numel(), torch.int64, buf.device)
        nb = max(16, self.D.fold_side_bytes(end - origin, halo))
        side = self._buf(("side", key), (nb + 7) // 8, torch.int64, buf.device)
        self.D.fold_range(buf, dst, origin, end, pos_base, fold_len, halo, side)
        return dst, side

    def total(self, side, span, halo, key=0):
        """16 bytes: the range's segmented total (int32 x 4)."""
        t = torch.empty(4, dtype=torch.int32, device=side.device)
        self.D.fold_range_total(side, span, halo, t)
        return t

    def patch(self, dst, origin, end, pos_base, fold_len, halo, side, prev):
        """The long-run patch with the totals of the ranges before (list, in order)."""
        pt = torch.cat(prev).contiguous() if prev else None
        self.D.fold_range_patch(dst, origin, end, pos_base, fold_len, halo, side, pt)

    def compact(self, chunk, d, key=0):
        n = chunk.numel() + d
        buf = self._buf(("cbuf", key), n, torch.int64, chunk.device)
        tmp = self._buf(("ctmp", key), n, torch.int64, chunk.device)
        return self.D.compact_range(chunk, d, 1.0, buf, tmp)

    def finish(self, out, coef):
        return self.D.sum_rows(out.view(1, -1), coef)

    def dp(self, out, sigma, clipping, n, seed):
        self.D.dp_noise(out, sigma, clipping, n, seed)


class VirtualRanks:
    """Every range lives in this process (the 1-GPU parity tests): exchanges are copies."""

    def __init__(self, world):
        self.world = world

    def swap(self, chunks, partner):
        return {r: chunks[partner(r)].clone() for r in chunks}

    def transpose(self, chunks, outs):
        w = self.world
        b = chunks[0].numel() // w
        for r in range(w):
            for q in range(w):
                outs[q][r * b:(r + 1) * b].copy_(chunks[r][q * b:(q + 1) * b])

    def neighbours(self, chunks, h, t, pads):
        w = self.world
        prev = {r: chunks[r - 1][-h:].clone() if r > 0 else pads(h, chunks[r]) for r in chunks}
        nxt = {r: chunks[r + 1][:t].clone() if r < w - 1 else pads(t, chunks[r]) for r in chunks}
        return prev, nxt

    def all_true(self, flag):
        return flag

    def gather_totals(self, tots):
        """Every range gets the totals of all ranges, in range order."""
        every = [tots[q] for q in range(self.world)]
        return {r: every for r in tots}

    def reduce(self, outs, root):
        out = outs[0].clone()
        for r in range(1, self.world):
            out += outs[r]
        return out

    def gather_lists(self, lists, root):
        """The ranges' lists concatenated in range order (on the root)."""
        return torch.cat([lists[r] for r in range(self.world)])


class DistRanks:
    """One range per process over torch.distributed (RCCL on the GPUs, gloo on CPU)."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world
        self._ready = False

    def ensure_init(self):
        """One full-group collective before the first batched P2P: with RCCL the first
        batch_isend_irecv of a group must include every rank, and pad skipping leaves
        the ranges past the live bound out of a pairwise stage."""
        if not self._ready:
            dist.barrier()
            self._ready = True

    @staticmethod
    def _run(ops):
        """ops: (send?, tensor, peer).  RCCL: one batched group; gloo (CPU tests, the
        one-GPU rehearsal) moves host copies of device tensors."""
        if not ops:
            return
        staged = dist.get_backend() == "gloo" and any(t.is_cuda for _, t, _ in ops)
        p2p, back = [], []
        for send, t, peer in ops:
            h = t.cpu() if (staged and send) else (torch.empty(t.shape, dtype=t.dtype) if staged else t)
            if staged and not send:
                back.append((h, t))
            p2p.append(dist.P2POp(dist.isend if send else dist.irecv, h, peer))
        for req in dist.batch_isend_irecv(p2p):
            req.wait()
        for h, t in back:
            t.copy_(h)

    def swap(self, chunks, partner):
        x = chunks[self.rank]
        theirs = torch.empty_like(x)
        p = partner(self.rank)
        self._run([(True, x, p), (False, theirs, p)])
        return {self.rank: theirs}

    def transpose(self, chunks, outs):
        """Block q of this range -> block `rank` of range q (one RCCL all-to-all: every
        xGMI link carries C/W records at once)."""
        x, out = chunks[self.rank], outs[self.rank]
        if dist.get_backend() == "gloo" and x.is_cuda:
            h = torch.empty(x.shape, dtype=x.dtype)
            dist.all_to_all_single(h, x.cpu())
            out.copy_(h)
        else:
            dist.all_to_all_single(out, x)

    def neighbours(self, chunks, h, t, pads):
        r, w, x = self.rank, self.world, chunks[self.rank]
        prev = torch.empty(h, dtype=x.dtype, device=x.device) if r > 0 else pads(h, x)
        nxt = torch.empty(t, dtype=x.dtype, device=x.device) if r < w - 1 else pads(t, x)
        ops = []
        if r > 0:
            ops += [(True, x[:t].contiguous(), r - 1), (False, prev, r - 1)]
        if r < w - 1:
            ops += [(True, x[-h:].contiguous(), r + 1), (False, nxt, r + 1)]
        self._run(ops)
        return {r: prev}, {r: nxt}

    def all_true(self, flag):
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def gather_totals(self, tots):
        """All ranks' 16-byte fold totals to every rank (one all_gather)."""
        x = tots[self.rank]
        staged = dist.get_backend() == "gloo" and x.is_cuda
        h = x.cpu() if staged else x
        parts = [torch.empty_like(h) for _ in range(self.world)]
        dist.all_gather(parts, h)
        if staged:
            parts = [p.to(x.device) for p in parts]
        return {self.rank: parts}

    def gather_lists(self, lists, root):
        """Variable-length lists to the root, concatenated in rank order: the counts go
        first (all_gather), the lists padded to the longest (one gather)."""
        x = lists[self.rank]
        staged = dist.get_backend() == "gloo" and x.is_cuda
        dev = "cpu" if (staged or not x.is_cuda) else x.device
        n = torch.tensor([x.numel()], dtype=torch.int64, device=dev)
        counts = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(counts, n)
        counts = [int(c.item()) for c in counts]
        width = max(1, max(counts))
        buf = torch.full((width,), -1, dtype=torch.int64, device=dev)
        buf[: x.numel()] = x.to(dev)
        parts = [torch.empty_like(buf) for _ in range(self.world)] if self.rank == root else None
        dist.gather(buf, parts, dst=root)
        if self.rank != root:
            return None
        out = torch.cat([parts[r][: counts[r]] for r in range(self.world)])
        return out.to(x.device)

    def reduce(self, outs, root):
        out = outs[self.rank]
        if dist.get_backend() == "gloo" and out.is_cuda:
            h = out.cpu()
            dist.reduce(h, dst=root, op=dist.ReduceOp.SUM)
            out.copy_(h)
        else:
            dist.reduce(out, dst=root, op=dist.ReduceOp.SUM)
        return out if self.rank == root else None


def distributed_network(chunks, world, M, ops, comm, mode=0, seed=0, exchange="transpose",
                        spare=None, valid=None):
    """The reference network (advanced.rs:147-176; mode 2: the keyed shuffle of
    nips19.rs:66-105) over M positions split into `world` ranges of C = M / world:
    every range runs stages up to C on its own, then each later stage does its steps
    j >= C across ranges (see index_sharded_advanced for the two exchanges; the
    transposed one needs only directions, so mode 2 always swaps pairwise) and its
    steps j < C inside each range.  Returns the chunks dict (ranges may have moved to
    the `spare` buffers).

    valid (None: unknown): positions >= valid hold identical pads.  A stage leaves every
    aligned 2^stage block of pads alone as it is, so a range sort runs on its live prefix
    only (a range of pads alone not at all), and a pairwise stage skips the ranges at or
    past roundup(valid, 2^stage) — a skipped range's partners lie in the same block, so
    both sides skip the exchange.  The transposed exchange mixes every range: its stages
    skip nothing.  Public sizes only: the network stays oblivious and bit-identical."""
    C = M // world
    clog, mlog = C.bit_length() - 1, M.bit_length() - 1
    assert 1 << clog == C and 1 << mlog == M
    vbound = M if valid is None else min(int(valid), M)
    if hasattr(comm, "ensure_init"):
        comm.ensure_init()  # every rank enters here; later stages may skip some ranks

    def live_from(stage):
        blk = 1 << stage
        return min((vbound + blk - 1) // blk * blk, M)

    for r, x in chunks.items():
        lo = r * C
        if lo >= vbound:
            continue  # pads alone
        ops.sort(x, lo, mode=mode, seed=seed, valid=None if vbound - lo >= C else vbound - lo)
    wlog = world.bit_length() - 1
    transpose = exchange == "transpose" and world > 1 and mode == 0
    if transpose:
        assert clog >= wlog
        spare = spare if spare is not None else {r: torch.empty_like(x) for r, x in chunks.items()}
        chunks = dict(chunks)
    for stage in range(clog + 1, mlog + 1):
        if transpose:
            comm.transpose(chunks, spare)
            chunks, spare = spare, chunks
            for r, x in chunks.items():  # transposed: global bits clog.. are local bits clog-wlog..
                ops.steps(x, 0, stage - wlog, stage - 1 - wlog, clog - wlog)
            comm.transpose(chunks, spare)
            chunks, spare = spare, chunks
        else:
            sf = live_from(stage)
            live = {r: x for r, x in chunks.items() if r * C < sf}
            for j in range(stage - 1, clog - 1, -1):
                bit = 1 << (j - clog)
                theirs = comm.swap(live, lambda q: q ^ bit) if live else {}
                for r, x in live.items():
                    ops.exchange(x, theirs[r], r * C, (r ^ bit) * C, stage, mode=mode, seed=seed)
                del theirs
        sf = M if transpose else live_from(stage)
        for r, x in chunks.items():
            if r * C < sf:
                ops.merge(x, r * C, stage, mode=mode, seed=seed)
    return chunks


def index_sharded_nips19(chunks, world, M, n_total, d, seed, ops=None, comm=None, root=0,
                         dp=None, valid=None):
    """nips19 (nips19.rs:18-63) by position range: `chunks` = the ranges of the padded
    array (records ++ Laplace dummies ++ pads, fltee_nips19_build_range with the same
    Laplace counts on every rank: counter-based, no exchange); the keyed shuffle runs
    as a distributed network (pairwise exchanges, mode 2), every rank runs
    safe_aggregate's selection on its range (its entries with idx < d, in position
    order), the lists are gathered to the root in rank order — the shuffled order — and
    the root adds each index's entries in that order (fltee_ordered_list_device), x
    1f32/n, then DP noise.  Bit-identical to one GPU's nips19.  valid = n·k + d·⌊T⌋ (the
    records and Laplace dummies in front of the pads) lets the network skip pad blocks."""
    assert world & (world - 1) == 0 and M % world == 0
    ops = ops if ops is not None else DeviceRangeOps()
    comm = comm if comm is not None else VirtualRanks(world)
    key = (seed ^ (seed >> 32)) & 0xFFFFFFFF  # the shuffle key of fltee_aggregate_device
    chunks = distributed_network(chunks, world, M, ops, comm, mode=2, seed=key, exchange="pairwise",
                                 valid=valid)
    lists = {r: ops.select(x, d) for r, x in chunks.items()}
    full = comm.gather_lists(lists, root)
    if full is None:
        return None
    out = ops.ordered(full, d, float(np.float32(1.0) / np.float32(n_total)))
    if dp is not None:
        ops.dp(out, dp["sigma"], dp["clipping"], n_total, dp.get("seed", 0))
    return out


def index_sharded_advanced(chunks, world, M, n_total, k, d, ops=None, comm=None, halo=None,
                           root=0, dp=None, exchange="transpose", spare=None):
    """Option B: `advanced` over the padded array of M = next_pow2(n_total*k + d)
    entries split into `world` ranges of C = M / world.  `chunks` maps a range index r
    to its C entries (positions [r*C, (r+1)*C), built by fltee_advanced_init_range);
    one entry per process under DistRanks, all of them under VirtualRanks.  The
    chunks are sorted in place.  Returns the averaged f32[d] on the root (None
    elsewhere); dp = dict(sigma, clipping, seed) adds the noise there (lib.rs:399-408).

    advanced.rs:39-113 step by step: the network (:147-176) = per-range stages up to
    C, then per stage the exchange steps (j >= C, partner r ^ j/C) and the range's
    own steps (j < C); the fold (:66-101) with fold_context(halo) + 16 records of the
    previous range in front and the next range's first records behind, then the
    long-run patch: every range's segmented total goes to the ranges after it, which
    finish the runs begun before them (runs of any length: bit for bit up to halo + 1
    entries, re-associated at the fold's walk boundaries beyond); the second
    sort's [0, d) prefix (:106-111, :32-34) = each range's compacted representatives,
    summed over the ranges by one reduce, then x 1f32/n (common.rs:14-19).

    exchange = "pairwise": every cross-range step swaps whole ranges with the partner
    (one xGMI link per pair, W = 8: six steps of C records).  "transpose" (default): per
    stage, one all-to-all swaps the rank bits of the position with the top log2 W local
    bits (block q of range r <-> block r of range q: contiguous blocks, no packing), the
    stage's cross-range steps then run locally as register passes
    (fltee_bitonic_range_steps_device; mode 0 only needs the direction, which is global
    bit `stage` = local bit stage - log2 W of the transposed range), and a second
    all-to-all restores the layout before the range's own steps.  Every link carries
    C/W records per all-to-all.  `spare` = {r: tensor like chunks[r]} reuses buffers."""
    assert world & (world - 1) == 0 and M % world == 0
    ops = ops if ops is not None else DeviceRangeOps()
    comm = comm if comm is not None else VirtualRanks(world)
    C = M // world
    chunks = distributed_network(chunks, world, M, ops, comm, exchange=exchange, spare=spare,
                                 valid=n_total * k + d)
    fold_len = n_total * k + d
    # one fold with halo n (or the caller's), fixed cost: a run of more than halo + 1
    # entries (a client repeated an index) is finished by the patch, no rerun
    h = n_total if halo is None else halo
    X = ops.fold_context(h) + 16  # the halo and the record in front of the first walk
    if X > C:
        raise ValueError(f"fold context {X} exceeds the range size {C}")
    prev, nxt = comm.neighbours(chunks, X, 16, ops.pads)
    folded, sides, tots = {}, {}, {}
    for r, x in chunks.items():
        buf = torch.cat([prev[r], x, nxt[r]])
        folded[r], sides[r] = ops.fold(buf, X, X + C, r * C - X, fold_len, h, key=r)
        tots[r] = ops.total(sides[r], C, h, key=r)
    every = comm.gather_totals(tots)
    for r, f in folded.items():
        ops.patch(f, X, X + C, r * C - X, fold_len, h, sides[r], every[r][:r])
    outs = {r: ops.compact(f[X:X + C], d, key=r) for r, f in folded.items()}
    out = comm.reduce(outs, root)
    if out is None:
        return None
    coef = float(np.float32(1.0) / np.float32(n_total))
    out = ops.finish(out, coef)
    if dp is not None:
        ops.dp(out, dp["sigma"], dp["clipping"], n_total, dp.get("seed", 0))
    return out

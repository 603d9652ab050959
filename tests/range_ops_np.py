"""numpy stand-ins for the HIP range pieces of position-sharded `advanced`
(include/fltee_agg.h, SURVEY §8e Option B), so the CPU tests can run
fltee.parallel.index_sharded_advanced — its order of steps and its exchanges —
without a GPU.  Each follows the reference network / fold literally
(advanced.rs:66-101,147-176), with global positions.  Test infrastructure only."""
import numpy as np
import torch

MASK = np.uint64(0xFFFFFFFF)
PAD = 0xFFFFFFFF


def _u(x):
    return x.numpy().view(np.uint64)


def _mix32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def step_key(seed, ilog, jlog):
    """shuffle_step_key of fl-tee_amd/csrc/common.h (the keyed comparator's per-step key)."""
    return _mix32(_mix32(seed) + ((ilog << 8) | jlog) * 0x9E3779B9)


def _cond2(lo, hi, l, mode, key):
    if mode == 0:
        return (lo & MASK) < (hi & MASK)
    h = ((l.astype(np.uint64) ^ np.uint64(key)) * np.uint64(0x9E3779B1)) & MASK
    return (h >> np.uint64(31)) != 0


def _step(a, pbase, ilog, jlog, mode=0, seed=0):
    """One step (stage 2^ilog, distance 2^jlog < len(a)) of advanced.rs:155-175 (mode 0)
    or of the keyed shuffle (mode 2)."""
    j = 1 << jlog
    x = np.arange(len(a) // 2, dtype=np.int64)
    l = ((x & ~(j - 1)) << 1) | (x & (j - 1))
    m = l + j
    asc = ((pbase + l) & (1 << ilog)) == 0
    al, am = a[l].copy(), a[m].copy()
    key = step_key(seed, ilog, jlog) if mode == 2 else 0
    sw = asc ^ _cond2(al, am, pbase + l, mode, key)
    a[l] = np.where(sw, am, al)
    a[m] = np.where(sw, al, am)


class NumpyRangeOps:
    def pads(self, n, like):
        return torch.full((n,), PAD, dtype=torch.int64)

    def fold_context(self, halo):
        return (halo + 15) // 16 * 16

    def sort(self, x, pos, mode=0, seed=0, valid=None):  # valid: the full network is the same
        a = _u(x)
        for ilog in range(1, len(a).bit_length()):
            for jlog in range(ilog - 1, -1, -1):
                _step(a, pos, ilog, jlog, mode, seed)

    def merge(self, x, pos, stage_log, mode=0, seed=0):
        a = _u(x)
        for jlog in range(len(a).bit_length() - 2, -1, -1):
            _step(a, pos, stage_log, jlog, mode, seed)

    def exchange(self, x, theirs, pos, pos_theirs, stage_log, mode=0, seed=0):
        a, b = _u(x), _u(theirs)
        lower = pos < pos_theirs
        lo, hi = (a, b) if lower else (b, a)
        p = min(pos, pos_theirs) + np.arange(len(a), dtype=np.int64)
        asc = (p & (1 << stage_log)) == 0
        jlog = (abs(pos - pos_theirs)).bit_length() - 1
        key = step_key(seed, stage_log, jlog) if mode == 2 else 0
        sw = asc ^ _cond2(lo, hi, p, mode, key)
        a[:] = np.where(sw, b, a)

    def safe_aggregate(self, x, d):
        """common.rs:25-35 on one range: g[idx] += val for idx < d, in position order."""
        a = _u(x)
        idx = (a & MASK).astype(np.int64)
        val = (a >> np.uint64(32)).astype(np.uint32).view(np.float32)
        out = np.zeros(d, np.float32)
        sel = idx < d
        np.add.at(out, idx[sel], val[sel])
        return torch.from_numpy(out)

    def select(self, x, d):
        a = _u(x)
        return torch.from_numpy(a[(a & MASK) < d].view(np.int64).copy())

    def ordered(self, lst, d, coef):
        """common.rs:25-35 + 14-19 on the concatenated list: in-order f32 sums, x coef."""
        a = _u(lst)
        idx = (a & MASK).astype(np.int64)
        val = (a >> np.uint64(32)).astype(np.uint32).view(np.float32)
        out = np.zeros(d, np.float32)
        np.add.at(out, idx, val)
        return torch.from_numpy(out * np.float32(coef))

    def steps(self, x, pos, stage_log, step_top, step_bot):
        a = _u(x)
        for jlog in range(step_top, step_bot - 1, -1):
            _step(a, pos, stage_log, jlog)

    def fold(self, buf, origin, end, pos_base, fold_len, halo, key=0):
        """fo_fold (advanced.rs:66-101) over the buffer's global positions, one walk from
        local position 1 (the record in front of it tells whether the run there began
        before): the context in front makes the carry exact for every run of <= halo + 1
        entries; a run begun before the walk and ended in [origin, end) is left as a dummy
        and carried by the side record (the device's FoldSide, one walk per range here)."""
        s = _u(buf)
        out = s.copy()
        b, C = 1, end - origin
        hasprev = pos_base + b - 1 >= 0
        kprev = int(s[b - 1] & MASK) if hasprev else None
        started, pre_i, pre_v = False, 0, np.float32(0)
        in_head, unbroken, corr, piece, pfull = False, True, False, False, False
        ck, cs, pf_key, pk, pq = 0, np.float32(0), 0, 0, np.float32(0)
        for q in range(b, end + 1):
            g = pos_base + q
            ci = int(s[q] & MASK)
            cv = np.uint32(int(s[q] >> np.uint64(32))).view(np.float32)
            eq = started and ci == pre_i
            copy = g - 1 >= fold_len
            dmy = g < fold_len and eq
            hend = in_head and not copy and not dmy
            sup = hend and origin <= q - 1 < end
            if origin <= q - 1 < end:
                if copy:
                    out[q - 1] = s[q - 1]
                elif dmy or sup:
                    out[q - 1] = np.uint64(0xFFFFFFFF - (g - 1))
                else:
                    out[q - 1] = np.uint64(pre_i) | (np.uint64(np.float32(pre_v).view(np.uint32)) << np.uint64(32))
            if sup:
                corr, ck, cs = True, pre_i, pre_v
            in_head = in_head and not hend and not copy
            if g >= 0:
                if not started:
                    pf_key = ci
                    in_head = hasprev and ci == kprev
                else:
                    unbroken = unbroken and eq
                pre_v = np.float32(pre_v + cv) if eq else cv
                pre_i = ci
                started = True
            if q == b + C - 1 and started and g >= 0:
                piece, pfull, pk, pq = True, unbroken, pre_i, pre_v
        fl = (1 if piece else 0) | (2 if piece and pfull else 0) | (4 if corr else 0)
        side = np.array([pf_key, pk, np.float32(pq).view(np.uint32), fl, ck,
                         np.float32(cs).view(np.uint32)], dtype=np.uint32)
        return torch.from_numpy(out.view(np.int64).copy()), side

    def total(self, side, span, halo, key=0):
        return torch.from_numpy(np.array([side[0], side[1], side[2], side[3] & 3], np.uint32).view(np.int32))

    @staticmethod
    def _agg(t):
        a = np.asarray(t).view(np.uint32)
        return int(a[0]), int(a[1]), np.uint32(a[2]).view(np.float32), int(a[3]) & 3

    @staticmethod
    def _combine(x, y):
        if not x[3] & 1:
            return y
        if not y[3] & 1:
            return x
        full = bool(x[3] & 2) and bool(y[3] & 2) and x[1] == y[0]
        q = np.float32(x[2] + y[2]) if (y[3] & 2 and y[0] == x[1]) else y[2]
        return x[0], y[1], q, 1 | (2 if full else 0)

    def patch(self, dst, origin, end, pos_base, fold_len, halo, side, prev):
        run = (0, 0, np.float32(0), 0)
        for t in prev:
            run = self._combine(run, self._agg(t.numpy() if hasattr(t, "numpy") else t))
        if side[3] & 4 and run[3] & 1 and run[1] == int(side[4]):
            tot = np.float32(run[2] + np.uint32(side[5]).view(np.float32))
            v = np.uint64(int(side[4])) | (np.uint64(tot.view(np.uint32)) << np.uint64(32))
            dst[origin] = torch.tensor(np.array([v], np.uint64).view(np.int64)[0])

    def compact(self, chunk, d, key=0):
        a = _u(chunk)
        idx = (a & MASK).astype(np.int64)
        val = (a >> np.uint64(32)).astype(np.uint32).view(np.float32)
        out = np.zeros(d, np.float32)
        sel = idx < d
        out[idx[sel]] = val[sel]
        return torch.from_numpy(out)

    def finish(self, out, coef):
        return out * np.float32(coef)

    def dp(self, out, sigma, clipping, n, seed):
        raise NotImplementedError


def init_range(idx, val, d, pos, C):
    """Entries [pos, pos + C) of advanced's padded array (advanced.rs:116-142)."""
    nrec = len(idx)
    p = pos + np.arange(C, dtype=np.int64)
    out = np.full(C, PAD, dtype=np.uint64)
    rec = p < nrec
    out[rec] = idx[p[rec]].astype(np.uint64) | (val[p[rec]].view(np.uint32).astype(np.uint64) << np.uint64(32))
    ini = (p >= nrec) & (p < nrec + d)
    out[ini] = (p[ini] - nrec).astype(np.uint64)
    return torch.from_numpy(out.view(np.int64).copy())

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
        """fo_fold (advanced.rs:66-101) over the buffer's global positions, started
        fresh at its first position: the context in front makes the carry exact."""
        s = _u(buf)
        out = s.copy()
        pre_i = pre_v = None
        for q in range(len(s)):
            g = pos_base + q
            if g < 0 or g >= fold_len:
                continue
            ci, cv = int(s[q] & MASK), np.uint32(int(s[q] >> np.uint64(32))).view(np.float32)
            if pre_i is None:
                pre_i, pre_v = ci, cv
            else:
                if ci == pre_i:
                    out[q - 1] = np.uint64(0xFFFFFFFF - (g - 1))
                    pre_v = np.float32(pre_v + cv)
                else:
                    out[q - 1] = np.uint64(pre_i) | (np.uint64(pre_v.view(np.uint32)) << np.uint64(32))
                    pre_i, pre_v = ci, cv
            if g == fold_len - 1:
                out[q] = np.uint64(pre_i) | (np.uint64(np.float32(pre_v).view(np.uint32)) << np.uint64(32))
        return torch.from_numpy(out.view(np.int64)[origin:end].copy()), 0

    def ok(self, statuses):
        return True

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

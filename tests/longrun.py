"""Checks for `advanced` / alg 6 on uploads with runs longer than n + 1 entries (a client
repeating an index).  The enclave folds every run left to right in the sorted order
(advanced.rs:66-101); the device folds each run of <= halo + 1 entries the same way (bit
for bit) and finishes longer ones with a sum re-associated at its fold's walk boundaries
(k_fold.hip / k_compact.hip headers) — within north_star's tolerance: the per-index
re-association bound below (every partial sum of a run of c values is within
(c - 1) * 2^-24 * sum|v| of the exact sum, for either order)."""
import numpy as np

U = 2.0 ** -24


def run_stats(idx, val, d):
    """per index i < d: the run length (records + the initial entry), sum |v|, exact sum"""
    idx = np.asarray(idx, np.int64)
    val = np.asarray(val, np.float32).astype(np.float64)
    sel = idx < d
    cnt = np.bincount(idx[sel], minlength=d)[:d] + 1
    absum = np.zeros(d, np.float64)
    np.add.at(absum, idx[sel], np.abs(val[sel]))
    exact = np.zeros(d, np.float64)
    np.add.at(exact, idx[sel], val[sel])
    return cnt, absum, exact


def assert_advanced(out, ref, idx, val, d, n, lim=None):
    """out vs the oracle's `advanced` (ref), both x 1f32/n: bit for bit wherever the run
    has <= lim (= n + 1) entries, within the re-association bound elsewhere; returns the
    number of long runs."""
    cnt, absum, _ = run_stats(idx, val, d)
    lim = n + 1 if lim is None else lim
    short = cnt <= lim
    o = np.asarray(out, np.float32)
    r = np.asarray(ref, np.float32)
    assert np.isfinite(o).all()
    diff = np.flatnonzero(short & (o.view(np.uint32) != r.view(np.uint32)))
    assert diff.size == 0, f"{diff.size} short runs differ (first idx {diff[:5]})"
    o64, r64 = o.astype(np.float64), r.astype(np.float64)
    bound = 2 * (cnt - 1) * U * absum / n + 2 * U * np.abs(r64) + 1e-45
    over = np.flatnonzero(~short & (np.abs(o64 - r64) > bound))
    if over.size:
        _, _, exact = run_stats(idx, val, d)
        det = [(int(i), int(cnt[i]), float(o64[i]), float(r64[i]), float(exact[i] / n), float(bound[i]))
               for i in over[:5]]
        raise AssertionError(f"{over.size} long runs over the bound: (idx, entries, out, ref, "
                             f"exact, bound) {det}")
    return int((~short).sum())


def assert_near_exact(out, idx, val, d, n):
    """out (x 1f32/n) vs the exact (float64) per-index sums: within the bound every f32
    left fold obeys — the full-size property check where the oracle's network is too
    slow to run per case."""
    cnt, absum, exact = run_stats(idx, val, d)
    o = np.asarray(out, np.float32).astype(np.float64)
    want = exact / n
    bound = (cnt - 1) * U * absum / n + 2 * U * np.abs(want) + 1e-45
    over = np.flatnonzero(np.abs(o - want) > bound)
    assert over.size == 0, f"{over.size} indices over the bound (first {over[:5]})"

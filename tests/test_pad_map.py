"""The pad-only units the sorts by key skip inside a stage's mixed block (k_bitonic.hip
pad_map / pad_units), checked on the CPU against the network itself: the set of positions
holding pads is simulated step by step (advanced.rs:155-175: pair (l, l + j), swap iff
((l & i) == 0) ^ (key[l] < key[m]); pads carry the largest key), and every unit a launch
would skip must hold pads alone at the step it starts with.  The keyed shuffle (mode 2)
keeps the stage-block bound only."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "fl-tee_amd", "lib", "libfltee_agg.so")


def pad_units(mode, valid, mlog, pbase, ilog, jstep, sblog, uplog):
    from fltee import _lib as L
    out = np.zeros(3, np.uint32)
    L.lib().fltee_debug_pad_units(mode, valid, mlog, pbase, ilog, jstep, sblog, uplog,
                                  out.ctypes.data_as(ctypes.c_void_p))
    return [int(x) for x in out]


def step(pad, pbase, s, j):
    """One step of the network on the boolean pad map (pads = the largest keys)."""
    v = pad.reshape(-1, 2, 1 << j)
    a, b = v[:, 0, :].copy(), v[:, 1, :].copy()
    l0 = pbase + np.arange(v.shape[0], dtype=np.int64) * (2 << j)
    asc = (((l0 >> s) & 1) == 0)[:, None]
    v[:, 0, :] = np.where(asc, a & b, a | b)
    v[:, 1, :] = np.where(asc, a | b, a & b)


def skipped(u, nunits):
    live, hat, hlen = u
    keep = np.zeros(nunits, bool)
    keep[:live] = True
    keep[hat:hat + hlen] = False
    return ~keep


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
@pytest.mark.parametrize("mlog,pbase", [(10, 0), (12, 0), (11, 1 << 11), (9, 3 << 9)])
def test_pad_units_hold_pads_alone(mlog, pbase):
    from fltee import _lib as L
    M = 1 << mlog
    rng = np.random.default_rng(mlog * 31 + pbase)
    valids = sorted(set([1, M - 1, M // 2 + 1, M // 2 - 1, 3 * M // 4 + 5] +
                        [int(x) for x in rng.integers(1, M, 6)]))
    L.lib().fltee_debug_set_pad_skip(2)
    found_hole = found_fine = 0
    for valid in valids:
        pad = np.zeros(M, bool)
        pad[valid:] = True
        for s in range(1, mlog + 1):
            for j in range(s - 1, -1, -1):
                # units: register groups of 2^R (R = 1..3) and tiles over superblocks 2^sb
                for sblog in sorted({j + 1, min(mlog, j + 3), mlog}):
                    if sblog < j + 1:
                        continue
                    for uplog in (0, max(0, sblog - 4)):
                        u = pad_units(0, valid, mlog, pbase, s, j, sblog, uplog)
                        n = (M >> sblog) << uplog
                        sk = skipped(u, n)
                        # unit i lies in superblock i >> uplog
                        sb_pad = pad.reshape(-1, 1 << sblog).all(axis=1)
                        assert (sb_pad[np.nonzero(sk)[0] >> uplog]).all(), (valid, s, j, sblog, u)
                        # the stage-block bound is never coarser than before (level 1)
                        old = ((valid + (1 << s) - 1) >> s << s)
                        old_live = ((min(old, M) + (1 << sblog) - 1) >> sblog) << uplog if old < M else n
                        assert u[0] <= old_live
                        found_hole += u[2] > 0
                        found_fine += (u[0] - u[2]) < old_live
                step(pad, pbase, s, j)
        npad = M - valid  # sorted: pads at the end (a descending range: at the start)
        want = np.arange(M) >= valid if ((pbase >> mlog) & 1) == 0 else np.arange(M) < npad
        assert (pad == want).all()
    assert found_hole and found_fine


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_pad_units_mode2_and_levels():
    from fltee import _lib as L
    mlog, valid = 12, 1000
    try:
        # the keyed shuffle: stage blocks only (a pad's path is the secret permutation)
        L.lib().fltee_debug_set_pad_skip(2)
        assert pad_units(2, valid, mlog, 0, 12, 5, 6, 0) == [1 << 6, 0, 0]
        assert pad_units(2, valid, mlog, 0, 10, 5, 6, 0) == [1024 >> 6, 0, 0]
        fine = pad_units(0, valid, mlog, 0, 12, 5, 6, 0)
        assert fine[0] - fine[2] < 1 << 6
        L.lib().fltee_debug_set_pad_skip(1)
        assert pad_units(0, valid, mlog, 0, 12, 5, 6, 0) == [1 << 6, 0, 0]
        L.lib().fltee_debug_set_pad_skip(0)
        assert pad_units(0, valid, mlog, 0, 10, 5, 6, 0) == [1 << 6, 0, 0]
    finally:
        L.lib().fltee_debug_set_pad_skip(2)

"""The planned bitonic schedule (k_bitonic.hip plan_network), checked on the CPU: its
launches, replayed in order, run exactly the reference network's steps (advanced.rs:155-175:
stage i = T+1 .. M, steps j = i-1 .. 0, each once, in order), every tile launch has a shape
the kernels accept, and the last launch is the contiguous merge that can carry nips19's
selection sink.  The permutation itself is checked on the GPU (test_gpu_parity.py)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "fl-tee_amd", "lib", "libfltee_agg.so")


def plan(mlog, tlog, nt, rmax):
    from fltee import _lib as L
    buf = np.zeros(8 * 512, np.uint32)
    n = L.lib().fltee_debug_network_plan(mlog, tlog, nt, rmax, buf.ctypes.data_as(ctypes.c_void_p), 512)
    assert 0 < n <= 512
    return buf[: 8 * n].reshape(n, 8)


def old_launches(mlog, tlog, nt, rmax, minw=4):
    """stage_steps' schedule: per stage, the steps j >= T in register passes of <= rmax
    (or strided passes of up to tlog - minw when more), then one merge."""
    rs = tlog - minw
    count = 0
    for s in range(tlog + 1, mlog + 1):
        ng = s - tlog
        per = rs if rs > rmax else rmax
        count += -(-ng // per) + 1
    return count


CASES = [(20, 12, 512, 4), (27, 14, 1024, 6), (24, 14, 1024, 6), (21, 13, 512, 5), (22, 14, 1024, 6),
         (26, 14, 1024, 6), (16, 11, 512, 4), (13, 12, 512, 4), (29, 14, 1024, 6)]


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
@pytest.mark.parametrize("mlog,tlog,nt,rmax", CASES)
def test_plan_replays_the_network(mlog, tlog, nt, rmax):
    p = plan(mlog, tlog, nt, rmax)
    want = [(s, b) for s in range(tlog + 1, mlog + 1) for b in range(s - 1, -1, -1)]
    got = []
    for reg, ilog, jtop, R, ilog_a, a_top, ilog_b, wd in p.tolist():
        if reg:
            assert 1 <= R <= rmax and jtop + 1 >= R
            got += [(ilog, b) for b in range(jtop, jtop - R, -1)]
            continue
        wlog, dtile = wd & 0xFF, wd >> 8
        rows = tlog - wlog
        assert ilog_a or ilog_b
        if wlog < tlog:  # strided: W = 2^wlog consecutive records x 2^rows rows 2^dtile apart
            assert 4 <= wlog and (1 << wlog) <= nt and dtile >= wlog
        else:
            assert dtile == tlog and not ilog_b
        if ilog_a:
            assert a_top < wlog  # the tail runs on the consecutive bits
            got += [(ilog_a, b) for b in range(a_top, -1, -1)]
        if ilog_b:
            top = dtile + rows - 1
            assert top <= ilog_b - 1  # the row bits are steps of stage ilog_b
            got += [(ilog_b, b) for b in range(top, dtile - 1, -1)]
    assert got == want
    last = p[-1].tolist()
    assert last[0] == 0 and last[4] == mlog and last[5] == tlog - 1 and last[6] == 0
    assert len(p) <= old_launches(mlog, tlog, nt, rmax)


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_plan_saves_launches_at_the_config_sizes():
    assert len(plan(27, 14, 1024, 6)) < old_launches(27, 14, 1024, 6) == 29
    assert len(plan(20, 12, 512, 4)) < old_launches(20, 12, 512, 4) == 16

"""Where the metric's literal config (100 x MLP-MNIST, dense baseline) spends its launch-to-
launch spread: per input BUFFER, the median of each launch's own event time
(less an empty event pair's), over rounds that visit every buffer in turn (cold: the buffers
together exceed 1.5 x the 256 MiB Infinity Cache).  Layouts: separate allocations (as
bench.py's) and slices of one allocation at a given alignment.  The plain streaming read
(fltee_debug_read_floor) runs over the same buffers beside it, to tell a kernel effect from
a memory-system one.

    python scripts/dense_buffer_probe.py [rounds]
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/fl-tee_amd")
import bench  # noqa: E402
from fltee import _lib as L  # noqa: E402
from fltee import device as D  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    w = bench.WORKLOADS["mnist100"]
    n, d = w["n"], w["d"]
    nb = n * d * 8
    nbuf = int(1.5 * 256 * 2 ** 20 // nb) + 2
    lib = L.lib()
    out = torch.empty(d, dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    sink = torch.zeros(8192, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    D.reserve(w["alg"], n, d, d, dense=True)
    src = bench.make_records(torch, n, d, None, 1000, dev)

    def layouts():
        yield "separate", [src.clone() for _ in range(nbuf)], None
        for align in (2 ** 21, 2 ** 16, 4096):
            step = (nb + align - 1) // align * align
            big = torch.empty(step * nbuf // 8 + align, dtype=torch.int64, device=dev)
            base = (-big.data_ptr()) % align // 8
            views = []
            for b in range(nbuf):
                v = big[base + b * step // 8: base + b * step // 8 + nb // 8]
                v.copy_(src.view(torch.int64).view(-1))
                views.append(v)
            yield f"one_alloc_align{align}", views, big

    def ev_time(fn, order):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in order]
        torch.cuda.synchronize()
        for (a, b), i in zip(ev, order):
            a.record(stream)
            fn(i)
            b.record(stream)
        torch.cuda.synchronize()
        return np.array([a.elapsed_time(b) * 1e3 for a, b in ev])

    empty = np.median(ev_time(lambda i: None, range(200)))
    print(json.dumps(dict(empty_pair_us=round(float(empty), 3), nbuf=nbuf, mb=nb / 1e6)), flush=True)
    for name, bufs, _keep in layouts():
        order = [b for _ in range(rounds) for b in range(nbuf)]

        def agg(i):
            D.aggregate(w["alg"], bufs[i], n, d, d, out=out, dense=True, status=status)

        def rd(i):
            assert lib.fltee_debug_read_floor(C.c_void_p(bufs[i].data_ptr()), nb,
                                              C.c_void_p(sink.data_ptr()), 1024,
                                              C.c_void_p(stream.cuda_stream)) == 0

        for _ in range(2):
            for i in range(nbuf):
                agg(i)
        ta = ev_time(agg, order) - empty
        tr = ev_time(rd, order) - empty
        assert int(status.item()) == 0
        per = []
        for b in range(nbuf):
            sel = np.array(order) == b
            per.append(dict(buf=b, ptr_mod_2m=bufs[b].data_ptr() % 2 ** 21,
                            ptr_gb=round(bufs[b].data_ptr() / 2 ** 30, 3),
                            agg_p50=round(float(np.median(ta[sel])), 2),
                            read_p50=round(float(np.median(tr[sel])), 2)))
        print(json.dumps(dict(layout=name, agg_pct=np.percentile(ta, [10, 50, 90]).round(2).tolist(),
                              read_pct=np.percentile(tr, [10, 50, 90]).round(2).tolist(),
                              per_buffer=per)), flush=True)
        del bufs, _keep
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

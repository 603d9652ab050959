"""Small-payload ECALLs for a kernel trace: each (n, k, alg) runs `reps`
host-inclusive calls of ecall_secure_aggregation, the groups 50 ms apart so a trace splits
by time; one JSON line per group with the host wall times and the ECALL's phase timers.
    rocprofv3 --kernel-trace -d gpurun_out/x -o run -- python3 scripts/small_ecall_trace.py [reps] [n:k ...]"""
import json
import sys
import time

import numpy as np
import torch

sys.path[:0] = [".", "fl-tee_amd"]
from fltee import device as D  # noqa: E402
from fltee.ecalls import Enclave  # noqa: E402

ALGS = {"advanced": 1, "baseline": 3, "non_oblivious": 4, "path_oram": 5}
shapes = [(3, 508), (30, 508), (3, 5089), (300, 508), (30, 5089)]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
if len(sys.argv) > 2:
    shapes = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]]
d = 50890
dev = torch.device("cuda", 0)
E = Enclave(0)
fl = 7000
for n, k in shapes:
    ids = np.arange(1, n + 1, dtype=np.uint32)
    g = torch.Generator(device=dev).manual_seed(n * 7 + k)
    idx = torch.argsort(torch.rand(n, d, generator=g, device=dev), dim=1)[:, :k].to(torch.int64)
    vals = torch.randn(n, k, generator=g, device=dev) * 0.01
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
    cipher = torch.empty_like(rec)
    D.decrypt(ids, rec, k * 8, cipher)
    host = cipher.cpu().numpy().view(np.uint8)
    for name, a in ALGS.items():
        fl += 1
        assert E.ecall_fl_init(fl, ids, d, k, 1.12, 1.0, 0.1, 1.0, a, 0, 0) == (0, 0)
        walls, ph = [], []
        torch.cuda.synchronize()
        time.sleep(0.05)
        t_start = time.perf_counter()
        for r in range(reps + 1):
            assert E.ecall_start_round(fl, r, n)[:2] == (0, 0)
            t0 = time.perf_counter()
            st, rv, out, tt = E.ecall_secure_aggregation(fl, r, ids, host, d, k, a)
            w = time.perf_counter() - t0
            assert (st, rv) == (0, 0), (name, st, rv)
            if r:
                walls.append(w * 1e6)
                ph.append([float(x) * 1e3 for x in tt])
        p = np.mean(np.array(ph), axis=0)
        print(json.dumps(dict(n=n, k=k, alg=name, payload_bytes=n * k * 8, reps=reps,
                              wall_us_mean=float(np.mean(walls)), wall_us_min=float(np.min(walls)),
                              load_us=float(p[0]), decrypt_us=float(p[1]), aggregate_us=float(p[2]),
                              t_start=t_start)), flush=True)
E.destroy()

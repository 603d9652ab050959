"""Check the bench's extrapolated CPU baselines for C4 and C5 against full-size runs.

bench_legs.cpu_baseline_configs times nips19 (C4) at request k/8 and advanced (C5) at
1/16 of d and k, and scales by the networks' compare-exchange ratio, so that the default
bench stays within minutes.  This script runs both the sample and the full size once,
single-threaded (the enclave has one TCS), and writes the measured ratio beside the
predicted one:  python scripts/cpu_extrapolation_check.py [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402

from bench_legs import _net_cost, _sparse_weights, host_cpu  # noqa: E402


def timed(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r04",
                                                             "cpu_extrapolation_check.json")
    O.build()
    O.set_threads(1)
    rng = np.random.default_rng(1)
    res = {"host": host_cpu(), "threads": 1}
    # C4: nips19 with the reference's FxHash shuffle, request k/8 vs the full request k
    n, d, k = 300, 44964, 4496
    w = _sparse_weights(O, rng, n, d, k)
    ks = k // 8
    Ms = O.next_pow2(n * k + d * int(O.nips19_threshold(d, ks, n)))
    M = O.next_pow2(n * k + d * int(O.nips19_threshold(d, k, n)))
    ts = timed(lambda: O.nips19(ks, w, d, n, seed=7, reference_shuffle=True))
    tf = timed(lambda: O.nips19(k, w, d, n, seed=7, reference_shuffle=True))
    res["c4"] = dict(sample_M=Ms, M=M, sample_s=ts, full_s=tf, predicted_s=ts * _net_cost(M) / _net_cost(Ms),
                     predicted_ratio=_net_cost(M) / _net_cost(Ms), measured_ratio=tf / ts)
    print("c4", res["c4"], flush=True)
    # C5: advanced at 1/16 of d and k vs full size (1000 x 100K over 10M)
    n, d, k = 1000, 10_000_000, 100_000
    ds, ks = d // 16, k // 16
    idx = (rng.integers(0, ds, n)[:, None] + np.arange(ks)[None, :]) % ds
    w = O.as_weights(idx.reshape(-1).astype(np.uint32), rng.normal(0, 0.01, n * ks).astype(np.float32))
    Ms = O.next_pow2(n * ks + ds)
    ts = timed(lambda: O.advanced(ks, w, ds, n))
    del w
    idx = (rng.integers(0, d, n)[:, None] + np.arange(k)[None, :]) % d
    w = O.as_weights(idx.reshape(-1).astype(np.uint32), rng.normal(0, 0.01, n * k).astype(np.float32))
    del idx
    M = O.next_pow2(n * k + d)
    tf = timed(lambda: O.advanced(k, w, d, n))
    res["c5"] = dict(sample_M=Ms, M=M, sample_s=ts, full_s=tf, predicted_s=ts * _net_cost(M) / _net_cost(Ms),
                     predicted_ratio=_net_cost(M) / _net_cost(Ms), measured_ratio=tf / ts)
    print("c5", res["c5"], flush=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

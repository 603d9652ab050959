"""A/B of library builds: one child process per variant (environment assignments, usually
FLTEE_LIB=<an A/B build from scripts/ab_build.sh>), each timing bench.bench_workload.  The
parent never touches the GPU.  One JSON line per (workload, variant, repeat).

    python scripts/ab_env.py c5 FLTEE_LIB=fl-tee_amd/lib/ab/libfltee_agg_x.so
(the empty variant, the product library, always runs first and last)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys, torch
sys.path.insert(0, {root!r}); sys.path.insert(0, {root!r} + "/fl-tee_amd")
import bench
from fltee import device as D
import hashlib, numpy as np
from fltee import _lib as L
dev = torch.device("cuda", 0)
r = bench.bench_workload(torch, D, {w!r}, steps={steps}, warmup=5, device=dev)
# the output's bits, to check that the variants compute the same aggregate
wl = bench.WORKLOADS[{w!r}]
rec = bench.make_records(torch, wl["n"], wl["d"], wl["k"], 1000, dev)
kw = dict(dense=wl["k"] is None)
if wl.get("dp"):
    kw.update(seed=7)
out = D.aggregate(wl["alg"], rec, wl["n"], wl["k"] or wl["d"], wl["d"], **kw).cpu().numpy()
h = hashlib.sha256(out.view(np.uint32).tobytes()).hexdigest()[:16]
print("RESULT " + json.dumps(dict(kernel_ms=r["kernel_s"] * 1e3, passes=r["net"]["passes"], out_sha=h,
      build=L.lib().fltee_version().decode(),
      kernels={{k: round(v["ms"] / v["launches"] * 1e3, 1) for k, v in r["net"]["kernels"].items()}})))
"""


def main():
    w = sys.argv[1]
    steps = {"c3": 300, "c1": 300, "mnist100": 300}.get(w, 10)
    reps = int(os.environ.get("AB_REPS", "2"))
    variants = [""] + sys.argv[2:] + [""]
    for rep in range(reps):
        for v in variants:
            env = dict(os.environ)
            for kv in v.split():
                k, val = kv.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, w=w, steps=steps)],
                               env=env, capture_output=True, text=True, timeout=240)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            res = json.loads(line[-1][7:]) if line else dict(error=p.stderr[-400:])
            print(json.dumps(dict(workload=w, variant=v or "default", rep=rep, **res)), flush=True)
            if p.returncode != 0:
                sys.exit(p.returncode)


if __name__ == "__main__":
    main()

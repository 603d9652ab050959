"""The exp5 host-inclusive ECALL rows alone (bench_legs.bench_exp5), one JSON line per row:
    python scripts/exp5_probe.py [reps]"""
import json
import sys

import torch

sys.path[:0] = [".", "fl-tee_amd"]
import bench_legs  # noqa: E402
from fltee import device as D  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
res = bench_legs.bench_exp5(torch, D, torch.device("cuda", 0), reps=reps)
for r in res["rows"]:
    print(json.dumps(r), flush=True)

"""Host-inclusive ECALLs over a multi-GPU enclave id (fltee_device_init_multi) vs one GPU.

Run as a child process by bench.py's multi-GPU run (rank 0, the other ranks wait on a
host barrier), or by hand:  python scripts/ecall_multi_bench.py --devices 8
Prints one JSON object.  Each workload's ciphertext sits in pageable host memory, as
the Rust host hands it to ecall_secure_aggregation (server.rs:162-183); the same
payload goes through a one-GPU eid and through the N-GPU eid, whose outputs must be
bit-identical.  Times are the ECALL wall time and its execution_time_results
{load, decrypt, aggregate} (lib.rs:292-301,344-353,410-419 contract).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))

WORKLOADS = {
    # name: alg, n, d, k (None = dense)
    "ns_dense_baseline": (3, 100, 1_000_000, None),
    "c5_advanced": (1, 1000, 10_000_000, 100_000),
    "c4_nips19": (2, 300, 44964, 4496),
}


def make_cipher(torch, D, n, d, k, seed):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(seed)
    if k is None:
        vals = torch.randn(n, d, generator=g, device=dev) * 0.01
        idx = torch.arange(d, device=dev, dtype=torch.int64).expand(n, d)
    else:
        vals = torch.randn(n, k, generator=g, device=dev) * 0.01
        j = torch.arange(k, device=dev, dtype=torch.int64)
        off = torch.randint(0, d, (n, 1), generator=g, device=dev)
        idx = (off + j.unsqueeze(0)) % d
    rec = (idx | (vals.view(torch.int32).to(torch.int64) << 32)).reshape(-1).contiguous()
    ids = np.arange(n, dtype=np.uint32)
    cipher = torch.empty_like(rec)
    D.decrypt(ids, rec, (k or d) * 8, cipher)  # CTR: encryption == decryption
    torch.cuda.synchronize()
    host = cipher.cpu().numpy().view(np.uint8)
    del rec, cipher, vals, idx
    return ids, host


def run(E, fl, ids, host, alg, d, k, reps):
    n = len(ids)
    st, rv = E.ecall_fl_init(fl, ids, d, k, 1.12, 1.0, 0.1, 1.0, alg, 0, 0)
    assert (st, rv) == (0, 0), (st, rv)
    E.ecall_start_round(fl, 0, n)
    walls, phases, out = [], [], None
    for r in range(reps + 1):
        t0 = time.perf_counter()
        st, rv, o, tt = E.ecall_secure_aggregation(fl, r, ids, host, d, k, alg)
        wall = time.perf_counter() - t0
        assert (st, rv) == (0, 0), (st, rv)
        E.ecall_start_round(fl, r + 1, n)
        if r:  # the first call sizes the staging buffers (benchmark.rs:355-359 drops it too)
            walls.append(wall)
            phases.append(tt.tolist())
        out = o
    ph = np.mean(np.array(phases), axis=0)
    return out, dict(ms_per_call=float(np.mean(walls)) * 1e3, load_ms=ph[0] * 1e3,
                     decrypt_ms=ph[1] * 1e3, aggregate_ms=ph[2] * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", type=int, default=0, help="GPUs (0 = all visible)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--workloads", default=",".join(WORKLOADS))
    args = ap.parse_args()
    import torch

    from fltee import device as D
    from fltee.ecalls import Enclave, set_debug_seed
    visible = torch.cuda.device_count()
    n_dev = min(args.devices or visible, visible)
    n_dev = 1 << (n_dev.bit_length() - 1)  # ranges need a power of two
    torch.cuda.set_device(0)
    res = dict(devices=n_dev, visible=visible, unit="client-params/s", reps=args.reps,
               note="ecall_secure_aggregation with pageable host ciphertext, one eid over "
                    f"{n_dev} GPUs (fltee_device_init_multi) vs a one-GPU eid; outputs bit-identical")
    E1, EN = Enclave(0), Enclave(list(range(n_dev)))
    fl = 10
    for name in [w for w in args.workloads.split(",") if w]:
        alg, n, d, k = WORKLOADS[name]
        ids, host = make_cipher(torch, D, n, d, k, 7)
        kk = d if k is None else k
        row = dict(alg=alg, n=n, d=d, k=kk, payload_bytes=int(host.size))
        outs = {}
        for label, E in (("one_gpu", E1), (f"{n_dev}_gpus", EN)):
            set_debug_seed(0x5EED)  # same nips19 / DP draws on both eids
            fl += 1
            outs[label], t = run(E, fl, ids, host, alg, d, kk, args.reps)
            t["value"] = n * kk / (t["ms_per_call"] / 1e3)
            row[label] = t
        set_debug_seed(0)
        a, b = outs["one_gpu"], outs[f"{n_dev}_gpus"]
        row["bit_identical"] = bool(np.array_equal(a.view(np.uint32), b.view(np.uint32)))
        row["speedup"] = row["one_gpu"]["ms_per_call"] / row[f"{n_dev}_gpus"]["ms_per_call"]
        res[name] = row
        del host
    E1.destroy()
    EN.destroy()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

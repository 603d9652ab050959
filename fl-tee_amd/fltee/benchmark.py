"""`bin/bench` of the reference (secure_aggregation/app/src/benchmark.rs) over the C ABI.

The same command line (clap options, benchmark.rs:37-94), the same one-shot round
(benchmark.rs:96-243): synthetic clients, client-side encryption, ecall_fl_init,
ecall_start_round, the timed ECALL (alg 6: ecall_client_size_optimized_secure_aggregation),
the checksum print; trials averaged with trial 0 discarded (benchmark.rs:336-379); the
result table printed and written as CSV to results/<alg>-<d>-<k>-<c>-<UTC>.txt
(benchmark.rs:400-411).  Columns: Load, Decryption, Aggregation (the enclave's own
execution_time_results) and Total (host wall time around the ECALL), in seconds.

    PYTHONPATH=fl-tee_amd python -m fltee.benchmark -a advanced -d 50890 -k 5089 -c 10000 \\
        --sampling_ratio 0.3 -t 3

Differences: the synthetic draw is numpy's (rand 0.8's ChaCha StdRng is not available):
the same shape (k distinct indices of [0, d) per client, value = idx * 0.001), not the
same numbers.  Clients are encrypted on the GPU with the library's AES-CTR (the
reference's client uses C++ AES: the same cipher and key layout).
"""
import argparse
import csv
import datetime
import os
import time

import numpy as np

from . import _lib as L
from .ecalls import Enclave

ALGS = {"advanced": [1], "nips19": [2], "baseline": [3], "non_oblivious": [4], "path_oram": [5],
        "optimized": [6], "all": [1, 2, 3, 4, 5, 6]}
NAMES = {1: "advanced", 2: "nips19", 3: "baseline", 4: "non_oblivious", 5: "path_oram",
         6: "optimized"}


def create_opts():
    """benchmark.rs:37-94."""
    ap = argparse.ArgumentParser(prog="bench", description="Benchmark different oblivious aggregations")
    ap.add_argument("-c", "--num_of_clients", type=int, default=10)
    ap.add_argument("-d", "--num_of_parameters", type=int, default=100000)
    ap.add_argument("-k", "--num_of_sparse_parameters", type=int, default=1000)
    ap.add_argument("-a", "--aggregation_alg", default="non_oblivious", choices=sorted(ALGS))
    ap.add_argument("--sigma", type=float, default=1.12)
    ap.add_argument("--clipping", type=float, default=1.0)
    ap.add_argument("--alpha", type=float, default=0.1)
    ap.add_argument("--sampling_ratio", type=float, default=0.01)
    ap.add_argument("-t", "--trial", type=int, default=1)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--dp", action="store_true")
    ap.add_argument("--optimal_num_of_clients", type=int, default=0)
    ap.add_argument("--device", type=int, default=0, help="HIP device (replaces the enclave file)")
    ap.add_argument("--results", default="results", help="output directory of the CSV")
    return ap


def synthetic_clients(num_of_clients, d, k, seed=13):
    """benchmark.rs:286-297: client i gets k distinct indices of [0, d), val = idx * 0.001."""
    rng = np.random.default_rng(seed)
    idx = np.empty((num_of_clients, k), dtype=np.uint32)
    for i in range(num_of_clients):
        idx[i] = rng.choice(d, k, replace=False)
    val = idx.astype(np.float32) * np.float32(0.001)
    return idx, val


def encrypt_clients(idx, val, device):
    """Client-side AES-128-CTR of every client's serialized records (utils.rs:17-53), on
    the GPU: uint8 [num_of_clients, k*8] host array."""
    import torch

    from .client import encrypt_parameters
    from .device import pack_records
    c, k = idx.shape
    rec = torch.from_numpy(pack_records(idx.reshape(-1), val.reshape(-1))).to(f"cuda:{device}")
    enc = encrypt_parameters(rec, np.arange(c, dtype=np.uint32))
    return enc.cpu().numpy().reshape(c, k * 8)


def one_shot_secure_aggregation(enclave, alg, opts, idx, val, enc, verbose):
    """benchmark.rs:96-243 -> [load, decrypt, aggregation, total] seconds."""
    c, k = idx.shape
    d = opts.num_of_parameters
    ids = np.arange(c, dtype=np.uint32)
    st, rv = enclave.ecall_fl_init(0, ids, d, k, opts.sigma, opts.clipping, opts.alpha,
                                   opts.sampling_ratio, alg, opts.verbose, opts.dp)
    if (st, rv) != (L.SUCCESS, L.SUCCESS):
        raise RuntimeError(f"Error at ecall_fl_init ({st:#x}, {rv:#x})")
    sample_size = int(np.float32(opts.sampling_ratio) * np.float32(c))
    if opts.optimal_num_of_clients > sample_size:
        raise RuntimeError(f"optimal_num_of_clients is more than client size {sample_size}")
    st, rv, sampled = enclave.ecall_start_round(0, 0, sample_size)
    if (st, rv) != (L.SUCCESS, L.SUCCESS):
        raise RuntimeError(f"Error at ecall_start_round ({st:#x}, {rv:#x})")
    uploaded = np.ascontiguousarray(enc[sampled]).reshape(-1)
    t0 = time.perf_counter()
    if alg == 6:
        st, rv, out, times = enclave.ecall_client_size_optimized_secure_aggregation(
            0, 0, opts.optimal_num_of_clients, sampled, uploaded, d, k, alg)
    else:
        st, rv, out, times = enclave.ecall_secure_aggregation(0, 0, sampled, uploaded, d, k, alg)
    total = time.perf_counter() - t0
    if (st, rv) != (L.SUCCESS, L.SUCCESS):
        raise RuntimeError(f"Error at the aggregation ECALL ({st:#x}, {rv:#x})")
    if verbose:
        print(f"[Server] total execution time: {total:.6f} s")
        check = np.float32(0.0)
        for cid in sorted(set(sampled.tolist())):  # sequential f32 folds, as the Rust host does
            check = np.float32(check + np.cumsum(val[cid], dtype=np.float32)[-1])
        check = np.float32(check / np.float32(len(set(sampled.tolist()))))
        enclave = np.cumsum(out, dtype=np.float32)[-1]
        print(f"[CheckSum] enclave: {enclave} == raw: {check}")
    return [float(x) for x in times] + [total]


def main(argv=None):
    opts = create_opts().parse_args(argv)
    algs = ALGS[opts.aggregation_alg]
    c, d, k = opts.num_of_clients, opts.num_of_parameters, opts.num_of_sparse_parameters
    print(f"[FL settings] alg={opts.aggregation_alg} sigma={opts.sigma} clipping={opts.clipping} "
          f"alpha={opts.alpha} clients={c} sampling_ratio={opts.sampling_ratio} d={d} k={k}")
    idx, val = synthetic_clients(c, d, k)
    enc = encrypt_clients(idx, val, opts.device)
    header = ["Algorithm", "num_of_parameters", "num_of_sparse_parameters", "num_of_clients",
              "Load [s]", "Decryption [s]", "Aggregation [s]", "Total [s]"]
    rows = []
    print("[Server] init_enclave...")
    enclave = Enclave(opts.device)
    print(f"[Server] Init Enclave Successful {enclave.geteid()}!")
    try:
        for alg in algs:
            name = f"optimized-{opts.optimal_num_of_clients}" if alg == 6 else NAMES[alg]
            avg = np.zeros(4)
            for i in range(opts.trial + 1):
                print(f"------------------- start  {i + 1} / {opts.trial + 1} -------------------")
                res = one_shot_secure_aggregation(enclave, alg, opts, idx, val, enc, opts.verbose)
                print("---------------------- end -----------------------")
                if i >= 1:  # trial 0 is discarded: caches are cold (benchmark.rs:355-359)
                    avg += res
                if opts.verbose:
                    rows.append([f"[{i}]: {name}", d, k, c] + [f"{x:.8f}" for x in res])
            avg /= max(opts.trial, 1)
            rows.append([f"Avg w/o [0] ({opts.trial} trial): {name}", d, k, c] +
                        [f"{x:.8f}" for x in avg])
    finally:
        enclave.destroy()
    try:
        from tabulate import tabulate
        print(tabulate(rows, headers=header, tablefmt="grid"))
    except ImportError:
        for r in [header] + rows:
            print(" | ".join(str(x) for x in r))
    stamp = datetime.datetime.now(datetime.timezone.utc).strftime("%Y%m%d%H%M%SUTC")
    alg_name = (f"optimized-{opts.optimal_num_of_clients}" if opts.aggregation_alg == "optimized"
                else opts.aggregation_alg)
    os.makedirs(opts.results, exist_ok=True)
    path = os.path.join(opts.results, f"{alg_name}-{d}-{k}-{c}-{stamp}.txt")
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)
    print(f"[Server] results -> {path}")
    return rows


if __name__ == "__main__":
    main()

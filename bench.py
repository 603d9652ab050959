"""bench.py — device-resident aggregation throughput of the FL-TEE enclave path on MI355X.

Metric (BASELINE.json): aggregated params/sec (device-resident) = client-parameter
contributions folded into the aggregate per second, i.e. n*k records / step time,
summed over all GPUs.

Headline workload (`ns`, SURVEY §8 row NS / the north-star target): aggregation_alg
= baseline over 100 clients x 1,000,000 dense fp32 updates per GPU (records of
8 B = u32 idx + f32 val, 800 MB), averaged with 1f32/n.  Multi-GPU: one process
per GPU, the parameter range is sharded (each rank owns 1M parameters of every
client: weak scaling) and each step ends with an RCCL gather of the averaged
shards to rank 0 over xGMI (the response vector is assembled on the root).

Output: ONE compact JSON line, the last line of stdout (≤ 4 KB: the driver parses it
from an 8 KB tail), holding the contract keys, the roofline of the dominant kernel, a
bounded CPU-baseline sample of the oracle (the C restatement of the enclave's
`baseline`, 1 thread), the host-inclusive ECALL rate, the metric's literal MLP-MNIST
config and one-number summaries of the other BASELINE.json configs.  Everything the
legs measured in full (per-kernel blocks, exp5's 40 rows, reference_configs, the
per-config CPU baselines, the multi-GPU legs) goes to the detail file the line names
(`--detail`, default gpurun_out/bench_detail.json); the legs live in bench_legs.py.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ns] [--no-extra]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fl-tee_amd"))

from bench_legs import (ALG_NAMES, HBM_PEAK_GBS, WORKLOADS, algorithmic_bytes,  # noqa: E402
                        bench_c4_index_sharded, bench_c5_index_sharded, bench_c5_sharded,
                        bench_exp5, bench_next_rows, bench_oram_tree, bench_reference_configs, bench_workload,
                        bench_ns_strong, c_abi_multi_gpu, cpu_baseline_configs, cpu_baseline_sample,
                        dominant_kernel, e2e_sample, make_records, network_records,
                        read_floor, rocprof_kernel, traffic_from_profiles, _build_id)


LINE_MAX_BYTES = 4096  # the driver reads the last line from an 8 KB stdout tail


def _r(x, nd=4):
    """round for the compact line (significant digits)"""
    if x is None or isinstance(x, (bool, int, str)):
        return x
    return float(f"{x:.{nd}g}")


def compact_line(full):
    """The one stdout line: the contract keys and one-number summaries of every leg in
    `full` (the detail dict bench.py writes to its detail file).  Pure: tests build it
    from stubbed legs (tests/test_bench_line.py)."""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "build", "config")
    line = {k: full[k] for k in keys if k in full}
    line["value"] = _r(line.get("value"), 6)
    line["ms_per_step"] = _r(line.get("ms_per_step"), 5)
    rf = full.get("roofline")
    if rf:
        line["roofline"] = {k: _r(rf.get(k), 5) for k in
                            ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                             "kernel_ms", "algorithmic_bytes", "rocprof_avg_us", "read_floor_gbs",
                             "frac_of_floor")
                            if k in rf}
    cb = full.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = {k: _r(cb.get(k)) for k in ("value", "unit", "cores", "kind", "sample")}
        # cores = the threads the timed restatement used (the enclave had one TCS); the host
        # it ran on, beside it (north_star: "core count stated")
        host = cb.get("host") or {}
        line["cpu_baseline"]["host_cores"] = host.get("logical_cpus")
        line["cpu_baseline"]["host_cores_available"] = host.get("cpus_available_to_process")
        line["cpu_baseline"]["host_model"] = host.get("model")
    e2e = full.get("e2e_host_inclusive")
    if e2e:
        line["e2e_host_inclusive"] = {"value": _r(e2e["value"]), "ms_per_call": _r(e2e["ms_per_call"]),
                                      "h2d_gbs": _r(e2e["bytes_h2d"] / e2e["load_ms"] / 1e6)
                                      if e2e.get("load_ms") else None}
    lit = full.get("metric_literal_config")
    if lit:
        line["metric_literal_config"] = {
            "value": _r(lit["value"]), "kernel_ms": _r(lit["kernel_ms"]),
            "kernel_ms_median": _r(lit.get("kernel_ms_median")),
            "frac": _r(lit["roofline"]["frac"]), "trials": lit.get("trials"),
            "launch_ms_pct": {k: _r(v) for k, v in (lit.get("launch_ms_pct") or {}).items()}}
        rf = lit.get("read_floor")
        if rf:  # the same bytes read by a plain streaming kernel in the same run
            line["metric_literal_config"]["read_floor_ms"] = _r(rf["us"] / 1e3)
            line["metric_literal_config"]["frac_of_floor"] = _r(rf["us"] / 1e3 / lit["kernel_ms"], 3)
    ex = full.get("extra")
    if ex and full.get("n_gpus", 1) == 1:
        cpu = full.get("cpu_baseline_configs", {})
        cfg = {}
        for name, e in ex.items():
            s = {"ms": _r(e.get("kernel_ms"))}
            roof = e.get("roofline")
            if roof:
                s["net_frac"] = _r(roof.get("frac"), 3)
                dk = roof.get("dominant_kernel")
                if dk:
                    s["top"] = dk["kernel"]
                    s["top_frac"] = _r(dk.get("frac"), 3)
            if isinstance(cpu.get(name), dict) and cpu[name].get("gpu_speedup"):
                s["cpu_x"] = _r(cpu[name]["gpu_speedup"], 3)
            cfg[name] = s
        line["configs"] = cfg
    elif ex:  # N > 1: the sharded legs
        legs = {}
        for name, e in ex.items():
            if not isinstance(e, dict):
                continue
            if "error" in e:
                legs[name] = {"error": str(e["error"])[:120]}
                continue
            if name == "c_abi_multi_gpu":  # per workload: one-GPU eid vs the N-GPU eid
                legs[name] = {wl: {"ms_1": _r(r["one_gpu"]["ms_per_call"]),
                                   "ms_n": _r(r[f"{e['devices']}_gpus"]["ms_per_call"]),
                                   "bit_identical": r.get("bit_identical")}
                              for wl, r in e.items()
                              if isinstance(r, dict) and "one_gpu" in r and "devices" in e}
                continue
            s = {k: _r(e[k]) for k in ("ms_per_step", "value", "scaling") if k in e}
            for k in ("bit_identical", "ns_ms", "c5_ms", "c4_ms"):
                if k in e:
                    s[k] = _r(e[k])
            legs[name] = s
        line["legs"] = legs
        if full.get("extra_timed_out"):
            line["extra_timed_out"] = full["extra_timed_out"]
    rc = full.get("reference_configs")
    if rc:
        line["reference_speedup"] = {k: _r(v["speedup"], 3) for k, v in rc.items() if isinstance(v, dict)}
    e5 = full.get("exp5")
    if e5 and e5.get("rows"):
        sp = sorted(r["speedup"] for r in e5["rows"])
        line["exp5"] = {"rows": len(sp), "speedup_min": _r(sp[0], 3),
                        "speedup_median": _r(sp[len(sp) // 2], 3)}
    nr = full.get("next_rows")
    if nr:
        line["next_rows"] = {"aes_gbs": _r(nr["aes_ctr_decrypt"]["gbs"]),
                             "client_producers_ms": _r(nr["client_producers"]["ms"])}
    ot = full.get("oram_tree")
    if ot and ot.get("rows"):
        line["oram_tree"] = {f"n{r['n']}_k{r['k']}": {"ms": _r(r["ms"]), "accesses": r["accesses"],
                                                     "ref_x": _r(r["speedup"], 3)}
                             for r in ot["rows"]}
    if full.get("detail"):
        line["detail"] = full["detail"]
    return line


def emit(full, detail_path):
    """Write the detail file (best effort) and print the compact line last."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(full, f, indent=1)
            full["detail"] = os.path.relpath(os.path.abspath(detail_path), ROOT)
        except OSError as ex:
            full["detail"] = f"not written: {ex}"[:100]
    s = json.dumps(compact_line(full), separators=(",", ":"))
    if len(s) > LINE_MAX_BYTES:  # never lose the headline to an oversized summary
        keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline", "detail")
        s = json.dumps({k: v for k, v in compact_line(full).items() if k in keep},
                       separators=(",", ":"))
    print(s, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="ns", choices=sorted(WORKLOADS))
    ap.add_argument("--no-extra", action="store_true", help="skip the other configs")
    ap.add_argument("--extra", default="mnist30,mnist100,c1,c3,c4,c5")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-configs", action="store_true",
                    help="skip the per-config CPU baseline (about a minute of CPU)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-inclusive ECALL leg")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="where the full results go (the stdout line is a summary)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from fltee import device as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FLTEE_BENCH_BACKEND=gloo + FLTEE_BENCH_ONE_DEVICE=1 rehearse the N>1 code path
    # with every rank on cuda:0 (RCCL refuses two ranks on one GPU); the default is
    # RCCL with one GPU per rank.
    if os.environ.get("FLTEE_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("FLTEE_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    w = WORKLOADS[args.workload]
    n, d, k = w["n"], w["d"], w["k"]
    kk = d if k is None else k

    recs = [make_records(torch, n, d, k, 17 + 101 * rank + b, device) for b in range(3)]
    # double-buffered shard outputs: step i's RCCL gather (async, RCCL's own stream)
    # overlaps step i+1's kernel; step i+2 waits for it before reusing the buffer
    outs = [torch.empty(d, dtype=torch.float32, device=device) for _ in range(2)]
    status = torch.zeros(1, dtype=torch.int32, device=device)
    gathered = ([[torch.empty(d, dtype=torch.float32, device=device) for _ in range(world)]
                 for _ in range(2)] if (world > 1 and rank == 0) else None)
    works = {}
    kw = dict(dense=k is None, status=status)
    if w.get("dp"):
        kw.update(dp=True, sigma=1.12, clipping=1.0, seed=7)
    D.reserve(w["alg"], n, kk, d, **{x: y for x, y in kw.items() if x != "status"})
    stream = torch.cuda.current_stream()
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]

    def step(i, ev=None):
        b = i % 2
        if (i - 2) in works:
            works.pop(i - 2).wait()  # the stream waits for the gather that read outs[b]
        if ev is not None:
            ev[0].record(stream)
        D.aggregate(w["alg"], recs[i % 3], n, kk, d, out=outs[b], **kw)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:  # final RCCL step: averaged shards -> root over xGMI
            works[i] = dist.gather(outs[b], gathered[b] if rank == 0 else None, dst=0,
                                   async_op=True)

    def drain():
        for j in sorted(works):
            works.pop(j).wait()

    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    region[0].record(stream)
    for i in range(args.steps):
        # N = 1: the K launches run back to back and one event pair brackets them all
        # (per-launch event pairs would add their own gaps); N > 1: per-step pairs, since
        # the stream also waits for the gathers between the kernels
        step(args.warmup + i, kev[i] if world > 1 else None)
    region[1].record(stream)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        kern = sum(a.elapsed_time(b) for a, b in kev) / args.steps / 1e3
    else:
        kern = region[0].elapsed_time(region[1]) / args.steps / 1e3
    if world > 1:
        t = torch.tensor([elapsed, kern], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern = float(t[0]), float(t[1])
    assert int(status.item()) == 0, f"device status {int(status.item()):#x}"
    ms = elapsed / args.steps * 1e3
    value = world * n * kk / (elapsed / args.steps)
    algo_bytes = n * kk * 8 + d * 4  # records read + averaged output written, per launch
    del recs, gathered
    full = None
    if rank == 0:
        rp = rocprof_kernel(args.workload, "dense_accumulate_v")
        full = {
            "metric": "aggregated params/sec (device-resident), 100 clients x MLP-MNIST updates",
            "value": value, "unit": "client-params/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "build": _build_id(),
            "config": {"workload": (f"{args.workload}: " + w["desc"])[:90],
                       "value_is": "the north-star shape (SURVEY 8: 100 clients x 1M dense params "
                                   "per GPU); the metric's literal 100 x MLP-MNIST workload is "
                                   "metric_literal_config",
                       "alg": ALG_NAMES[w["alg"]], "n_clients": n,
                       "d_per_gpu": d, "k": kk, "record_bytes": 8,
                       "parallelism": f"param-range shard x{world}" +
                                      (f" + {backend} gather to rank 0" if world > 1 else ""),
                       "timing": "value: host wall, barrier+sync bracketed; roofline: HIP events "
                                 "on the launch stream"},
            "roofline": {"bound": "hbm", "achieved": algo_bytes / kern / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": algo_bytes / kern / 1e9 / HBM_PEAK_GBS,
                         "traffic": traffic_from_profiles(args.workload),
                         "kernel": "dense_accumulate_v", "algorithmic_bytes": algo_bytes,
                         "kernel_ms": kern * 1e3,
                         "rocprof_avg_us": rp["avg_us"] if rp else None,
                         "rocprof_source": rp["source"] if rp else None},
        }
    if world > 1 and not args.no_extra:
        # Every sharded leg runs under a watchdog: if the legs overrun the budget (a stuck
        # collective), rank 0 prints the line with what finished and every rank exits, so
        # the headline measurement above is never lost to an extra.
        sharded = {}
        if rank == 0:
            full["extra"] = sharded
        budget = float(os.environ.get("FLTEE_BENCH_EXTRA_BUDGET_S", "420"))
        t_extra = time.monotonic()
        state = {"leg": None, "printed": False}
        lock = threading.Lock()
        disarm = threading.Event()

        def watchdog():
            if disarm.wait(budget):
                return  # the extras finished in time
            with lock:
                if rank == 0 and not state["printed"]:
                    full["extra_timed_out"] = state["leg"]
                    emit(full, args.detail)
                    state["printed"] = True
            os._exit(3)  # the headline line is printed, but a stuck leg is a failure

        threading.Thread(target=watchdog, daemon=True).start()
        xsteps = max(3, args.steps // 10)
        legs = [("ns_strong", lambda: bench_ns_strong(torch, D, dist, world, rank, device,
                                                      steps=max(10, args.steps), warmup=3)),
                ("c5_sharded", lambda: bench_c5_sharded(
                    torch, D, dist, world, rank, device, steps=xsteps, warmup=1))]
        if world & (world - 1) == 0:
            legs += [
                ("c5_index_sharded", lambda: bench_c5_index_sharded(
                    torch, D, dist, world, rank, device, steps=xsteps, warmup=1)),
                ("c5_index_sharded_pairwise", lambda: bench_c5_index_sharded(
                    torch, D, dist, world, rank, device, steps=xsteps, warmup=1,
                    exchange="pairwise")),
                ("c4_index_sharded", lambda: bench_c4_index_sharded(
                    torch, D, dist, world, rank, device, steps=xsteps, warmup=1))]
        if os.environ.get("FLTEE_BENCH_NO_CABI") != "1":
            # the C-ABI multi-GPU eid first (its own share of the budget, so the sharded legs
            # cannot crowd it out), in a child of rank 0 while every rank waits on a host
            # (gloo) barrier with its cached HBM released
            state["leg"] = "c_abi_multi_gpu"
            hostpg = dist.new_group(backend="gloo")
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            dist.barrier(group=hostpg)
            if rank == 0:
                sharded["c_abi_multi_gpu"] = c_abi_multi_gpu(world, timeout=max(60.0, 0.45 * budget))
            dist.barrier(group=hostpg)
        for name, fn in legs:
            state["leg"] = name
            sharded[name] = fn()
        state["leg"] = None
        disarm.set()
        if rank == 0:
            with lock:
                if not state["printed"]:
                    emit(full, args.detail)
                    state["printed"] = True
        dist.destroy_process_group()
        return

    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            full["cpu_baseline"] = cpu_baseline_sample(d, n, args.cpu_seconds)
        if world == 1 and not args.no_e2e and k is None:
            full["e2e_host_inclusive"] = e2e_sample(torch, D, n, d, device)
        if world == 1 and not args.no_extra:
            full["extra"] = run_config_legs(torch, D, device, args)
            # the metric's literal configuration (100 clients x MLP-MNIST, dense baseline),
            # inputs rotated through > 1.5 x the Infinity Cache so every launch reads HBM;
            # 3 trials, each warming every rotating buffer once: best and median reported
            trials = sorted((bench_workload(torch, D, "mnist100", steps=max(20, args.steps),
                                            warmup=12, device=device, cold=True, per_launch=True)
                             for _ in range(3)), key=lambda r: r["kernel_s"])
            lit = trials[0]
            # the spread of single launches: every trial's per-launch event
            # times, p10 / p50 / p90
            lts = np.array([x for t in trials for x in t.get("launch_ms", [])])
            pct = {f"p{q}": float(np.percentile(lts, q)) for q in (10, 50, 90)} if lts.size else {}
            floor = read_floor(torch, lit["bytes"], device)
            full["metric_literal_config"] = dict(
                workload=WORKLOADS["mnist100"]["desc"], value=lit["rate"], unit="client-params/s",
                kernel_ms=lit["kernel_s"] * 1e3, kernel_ms_median=trials[1]["kernel_s"] * 1e3,
                launch_ms_pct=pct, launches=int(lts.size),
                kernel_ms_trials=[t["kernel_s"] * 1e3 for t in trials],
                input_buffers=lit["nbuf"], trials=len(trials),
                roofline=dict(bound="hbm", achieved=lit["bytes"] / lit["kernel_s"] / 1e9,
                              peak=HBM_PEAK_GBS, unit="GB/s",
                              frac=lit["bytes"] / lit["kernel_s"] / 1e9 / HBM_PEAK_GBS,
                              frac_median=lit["bytes"] / trials[1]["kernel_s"] / 1e9 / HBM_PEAK_GBS,
                              algorithmic_bytes=lit["bytes"], kernel="dense_accumulate_w",
                              note="cold: inputs rotated over > 1.5 x 256 MiB; best of the trials "
                                   "(kernel_ms) and their median (kernel_ms_median)"),
                read_floor=floor)
            # the headline kernel against a plain streaming read of its own 804 MB, same run:
            # the practical ceiling beside the 8 TB/s peak
            if "roofline" in full:
                nsf = read_floor(torch, algo_bytes, device, reps=2, steps=20)
                full["roofline"]["read_floor_gbs"] = nsf["gbs"]
                full["roofline"]["frac_of_floor"] = nsf["us"] / 1e6 / kern
            if not args.no_cpu_baseline and not args.no_cpu_configs:
                gms = {nm: e["kernel_ms"] for nm, e in full["extra"].items()}
                full["cpu_baseline_configs"] = cpu_baseline_configs(gms)
            full["reference_configs"] = bench_reference_configs(torch, D, device)
            full["exp5"] = bench_exp5(torch, D, device)
            full["next_rows"] = bench_next_rows(torch, D, device)
            full["oram_tree"] = bench_oram_tree(torch, D, device)
        emit(full, args.detail)
    if world > 1:
        dist.destroy_process_group()


def run_config_legs(torch, D, device, args):
    """The other BASELINE.json configs on one GPU, device-resident: kernel time per
    aggregate and, for the oblivious paths, the network roofline with its dominant kernel."""
    extra = {}
    for name in [x for x in args.extra.split(",") if x]:
        wl = WORKLOADS[name]
        small = wl["n"] * (wl["k"] or wl["d"]) * 8 < 100e6  # < 100 MB: more launches
        ksteps = max(10, args.steps * 2) if small else max(5, args.steps // 5)
        r = bench_workload(torch, D, name, steps=ksteps, warmup=2 + ksteps // 10, device=device)
        extra[name] = dict(desc=WORKLOADS[name]["desc"], alg=r["alg"], n=r["n"], d=r["d"],
                           k=r["k"], ms_per_step=r["wall_s"] * 1e3 / ksteps,
                           kernel_ms=r["kernel_s"] * 1e3, value=r["rate"], unit="client-params/s")
        M = network_records(wl)
        if M:  # the oblivious paths: their network traffic, not the useful bytes
            nb = r["net"]["bytes"]
            alg_b = algorithmic_bytes(wl)
            roof = dict(bound="hbm", network_passes=r["net"]["passes"], network_bytes=nb,
                        network_records=M, achieved=nb / r["kernel_s"] / 1e9, peak=HBM_PEAK_GBS,
                        unit="GB/s", frac=nb / r["kernel_s"] / 1e9 / HBM_PEAK_GBS,
                        algorithmic_bytes=alg_b, algorithmic_gbs=alg_b / r["kernel_s"] / 1e9,
                        note="network bytes = read + write of the live (not pad-only) part of the "
                             "array per streaming pass (launch-side accounting); achieved = those "
                             "bytes / the aggregate's event time; algorithmic bytes per SURVEY 8(d)")
            dk = dominant_kernel(r["net"])
            if dk:
                dk["share_of_aggregate"] = dk["avg_us"] * dk["launches"] / (r["kernel_s"] * 1e6)
                rp = rocprof_kernel(name, dk["kernel"])
                if rp:
                    dk["rocprof"] = rp
                tr = traffic_from_profiles(f"{name}:{dk['kernel']}")
                dk["traffic"] = tr
                if tr:
                    dk["traffic_over_launch_bytes"] = tr / dk["bytes_per_launch"]
                roof["dominant_kernel"] = dk
            roof["kernels"] = r["net"]["kernels"]
            extra[name]["roofline"] = roof
    return extra


if __name__ == "__main__":
    main()

"""bench.py's stdout contract: the LAST line is one compact JSON object the driver can
parse from its 8 KB stdout tail (round 3's 21 KB line was not parsed: BENCH_r03.parsed
null).  Built here from stubbed legs — the full results of a real round-3 run
(profiles/r03/head_i/bench.json, every leg present) and a synthetic N>1 run — without a
GPU; the reference's harness likewise prints one compact result per run
(secure_aggregation/app/src/benchmark.rs:336-411)."""
import copy
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CONTRACT = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}
ROOFLINE = {"bound", "achieved", "peak", "unit", "frac", "traffic"}
CPU = {"value", "unit", "cores", "kind", "sample"}


def _full_n1():
    with open(os.path.join(ROOT, "profiles", "r03", "head_i", "bench.json")) as f:
        return json.load(f)


def _full_n8():
    full = {k: v for k, v in _full_n1().items() if k in CONTRACT | {"build", "roofline"}}
    full["n_gpus"] = 8
    leg = dict(desc="x" * 300, alg="advanced", n=1000, d=10_000_000, k=100_000, M=2 ** 27,
               range_records=2 ** 24, ms_per_step=3.2, value=3.1e10, unit="client-params/s",
               scaling="strong")
    full["extra"] = {"ns_strong": dict(leg, bit_identical=True),
                     "c5_sharded": dict(leg), "c5_index_sharded": dict(leg),
                     "c5_index_sharded_pairwise": dict(leg), "c4_index_sharded": dict(leg),
                     "c_abi_multi_gpu": dict(devices=8, visible=8, note="n" * 300, **{
                         wl: {"alg": 1, "payload_bytes": 1, "one_gpu": {"ms_per_call": 30.0},
                              "8_gpus": {"ms_per_call": 9.0}, "bit_identical": True,
                              "speedup": 3.3} for wl in ("ns", "c5", "c4")})}
    return full


@pytest.mark.parametrize("make", [_full_n1, _full_n8])
def test_line_is_compact_and_complete(make, tmp_path, capsys):
    full = make()
    assert len(json.dumps(full)) > 8000 or full["n_gpus"] > 1  # the detail is the big part
    bench.emit(full, str(tmp_path / "detail.json"))
    out = capsys.readouterr().out.strip().splitlines()
    last = out[-1]
    assert len(last.encode()) <= bench.LINE_MAX_BYTES
    line = json.loads(last)
    assert CONTRACT <= set(line)
    assert ROOFLINE <= set(line["roofline"])
    assert 0 < line["roofline"]["frac"] < 1
    if line["n_gpus"] == 1:
        assert CPU <= set(line["cpu_baseline"])
        # the threads used, and the host's core count and model beside them
        cb = line["cpu_baseline"]
        assert cb["cores"] == 1 and cb["host_cores"] >= cb["cores"] and cb["host_model"]
        for key in ("e2e_host_inclusive", "metric_literal_config", "configs", "exp5"):
            assert key in line
        assert {"c3", "c4", "c5"} <= set(line["configs"])
    else:
        assert line["legs"]["ns_strong"]["bit_identical"] is True
        assert line["legs"]["ns_strong"]["scaling"] == "strong"
        assert line["legs"]["c_abi_multi_gpu"]["c5"] == {"ms_1": 30.0, "ms_n": 9.0,
                                                         "bit_identical": True}
    # the detail file holds everything, and the line names it
    with open(tmp_path / "detail.json") as f:
        detail = json.load(f)
    assert set(detail) >= set(make()) - {"detail"}
    assert line["detail"].endswith("detail.json")


def test_oversized_summary_falls_back_to_headline(tmp_path, capsys):
    full = _full_n1()
    full["extra"] = {f"c{i}": copy.deepcopy(full["extra"]["c5"]) for i in range(200)}
    bench.emit(full, str(tmp_path / "d.json"))
    last = capsys.readouterr().out.strip().splitlines()[-1]
    assert len(last.encode()) <= bench.LINE_MAX_BYTES
    line = json.loads(last)
    assert CONTRACT <= set(line) and "roofline" in line and "cpu_baseline" in line


def test_unwritable_detail_still_prints(capsys):
    full = _full_n1()
    bench.emit(full, "/proc/no/such/dir/detail.json")
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["detail"].startswith("not written")


def test_rocprof_cross_check_reads_the_newest_round():
    """bench_legs.rocprof_kernel takes the newest committed rocprofv3 summary of a config
    (it read round 4's while round 5's existed)."""
    import glob

    import bench_legs
    rounds = sorted(os.path.basename(os.path.dirname(p)) for p in
                    glob.glob(os.path.join(ROOT, "profiles", "r0*", "ns_kernel_stats.csv")))
    rp = bench_legs.rocprof_kernel("ns", "dense_accumulate_v")
    assert rp is not None and rounds
    assert rp["source"] == os.path.join("profiles", rounds[-1], "ns_kernel_stats.csv")

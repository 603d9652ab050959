"""fltee.benchmark: the reference's `bin/bench` (benchmark.rs) over the C ABI, every
algorithm at a small size: table rows, CSV file, checksum line."""
import csv
import os

import pytest

pytestmark = pytest.mark.gpu


def test_bench_cli_all_algorithms(tmp_path, capsys):
    from fltee import benchmark
    rows = benchmark.main(["-a", "all", "-c", "20", "-d", "1000", "-k", "50", "--sampling_ratio",
                           "0.5", "-t", "1", "-v", "--optimal_num_of_clients", "5",
                           "--results", str(tmp_path)])
    avg = [r for r in rows if r[0].startswith("Avg")]
    assert [r[0].split(": ")[1] for r in avg] == ["advanced", "nips19", "baseline", "non_oblivious",
                                                  "path_oram", "optimized-5"]
    for r in avg:
        load, dec, agg, total = (float(x) for x in r[4:])
        assert min(load, dec, agg) >= 0 and total > 0
    out = capsys.readouterr().out
    assert out.count("[CheckSum]") == 12  # verbose: every trial of every algorithm
    files = os.listdir(tmp_path)
    assert len(files) == 1 and files[0].startswith("all-1000-50-20-")
    with open(tmp_path / files[0]) as f:
        got = list(csv.reader(f))
    assert got[0][4:] == ["Load [s]", "Decryption [s]", "Aggregation [s]", "Total [s]"]
    assert len(got) == 1 + len(rows)


def test_bench_cli_checksum_matches(capsys, tmp_path):
    """non_oblivious average == the raw f32 average of the sampled clients (the printed
    CheckSum line of benchmark.rs:226-239), to f32 summation-order tolerance."""
    from fltee import benchmark
    benchmark.main(["-a", "non_oblivious", "-c", "10", "-d", "500", "-k", "40", "--sampling_ratio",
                    "1.0", "-t", "1", "-v", "--results", str(tmp_path)])
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("[CheckSum]")]
    assert lines
    for ln in lines:
        a, b = ln.split("enclave: ")[1].split(" == raw: ")
        assert abs(float(a) - float(b)) <= 1e-4 * max(1.0, abs(float(b)))

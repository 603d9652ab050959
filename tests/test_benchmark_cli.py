"""Host logic of fltee.benchmark (benchmark.rs) on CPU: options, the trial loop (trial 0
discarded, benchmark.rs:355-359), the per-alg rows, the CSV name and layout
(benchmark.rs:400-411), with a stub enclave standing in for the HIP library."""
import csv
import os

import numpy as np
import pytest

from fltee import _lib as L
from fltee import benchmark


class StubEnclave:
    calls = []

    def __init__(self, device=0):
        self.eid = 7

    def geteid(self):
        return self.eid

    def destroy(self):
        pass

    def ecall_fl_init(self, fl_id, ids, d, k, sigma, clipping, alpha, ratio, alg, verbose, dp):
        self.d, self.alg = d, alg
        return L.SUCCESS, L.SUCCESS

    def ecall_start_round(self, fl_id, round_, sample_size):
        return L.SUCCESS, L.SUCCESS, np.arange(sample_size, dtype=np.uint32)

    def _agg(self, ids, enc, d, k, alg, batch=None):
        StubEnclave.calls.append((alg, len(ids), len(enc), batch))
        t = float(len(StubEnclave.calls))
        return L.SUCCESS, L.SUCCESS, np.zeros(d, np.float32), np.array([t, 2 * t, 3 * t], np.float32)

    def ecall_secure_aggregation(self, fl_id, round_, ids, enc, d, k, alg):
        return self._agg(ids, enc, d, k, alg)

    def ecall_client_size_optimized_secure_aggregation(self, fl_id, round_, batch, ids, enc, d, k, alg):
        return self._agg(ids, enc, d, k, alg, batch)


@pytest.fixture
def stubbed(monkeypatch):
    StubEnclave.calls = []
    monkeypatch.setattr(benchmark, "Enclave", StubEnclave)
    monkeypatch.setattr(benchmark, "encrypt_clients",
                        lambda idx, val, device: np.zeros((idx.shape[0], idx.shape[1] * 8), np.uint8))
    return StubEnclave


def test_options_match_benchmark_rs():
    o = benchmark.create_opts().parse_args([])
    assert (o.num_of_clients, o.num_of_parameters, o.num_of_sparse_parameters) == (10, 100000, 1000)
    assert o.aggregation_alg == "non_oblivious" and o.trial == 1
    assert (o.sigma, o.clipping, o.alpha, o.sampling_ratio) == (1.12, 1.0, 0.1, 0.01)
    with pytest.raises(SystemExit):
        benchmark.create_opts().parse_args(["-a", "bubble"])


def test_synthetic_clients_shape():
    idx, val = benchmark.synthetic_clients(5, 100, 10)
    assert idx.shape == (5, 10) and all(len(set(r.tolist())) == 10 for r in idx)
    assert (idx < 100).all() and np.array_equal(val, idx.astype(np.float32) * np.float32(0.001))


def test_trials_rows_and_csv(stubbed, tmp_path):
    rows = benchmark.main(["-a", "all", "-c", "20", "-d", "100", "-k", "10", "--sampling_ratio",
                           "0.5", "-t", "2", "--optimal_num_of_clients", "4",
                           "--results", str(tmp_path)])
    # 6 algorithms x (trial + 1) ECALLs, sample of 10 clients x 10 records x 8 B each
    assert [c[0] for c in stubbed.calls] == [a for a in (1, 2, 3, 4, 5, 6) for _ in range(3)]
    assert all(c[1] == 10 and c[2] == 10 * 10 * 8 for c in stubbed.calls)
    assert [c[3] for c in stubbed.calls if c[0] == 6] == [4, 4, 4]
    assert len(rows) == 6 and rows[0][0] == "Avg w/o [0] (2 trial): advanced"
    assert rows[-1][0] == "Avg w/o [0] (2 trial): optimized-4"
    # average of trials 1 and 2 of the first alg: load = (2 + 3) / 2
    assert float(rows[0][4]) == pytest.approx(2.5)
    files = os.listdir(tmp_path)
    assert len(files) == 1 and files[0].startswith("all-100-10-20-") and files[0].endswith("UTC.txt")
    with open(tmp_path / files[0]) as f:
        got = list(csv.reader(f))
    assert got[0] == ["Algorithm", "num_of_parameters", "num_of_sparse_parameters", "num_of_clients",
                      "Load [s]", "Decryption [s]", "Aggregation [s]", "Total [s]"]
    assert len(got) == 7


def test_optimal_num_of_clients_above_sample_panics(stubbed, tmp_path):
    with pytest.raises(RuntimeError, match="more than client size"):
        benchmark.main(["-a", "optimized", "-c", "10", "-d", "100", "-k", "10", "--sampling_ratio",
                        "0.5", "--optimal_num_of_clients", "6", "--results", str(tmp_path)])

"""The proto/secure_aggregation.proto wire and the gRPC front end (fltee.wire,
fltee.grpc_server) — SURVEY §8f row 3.

Fixtures (tests/golden/wire.npz) are messages serialised by the reference's own
generated src/secure_aggregation_pb2.py (tests/golden/make_fixtures.py).  CPU
tests: byte-identical encoding, decoding, and a Start -> Aggregate round trip over
a real localhost gRPC channel with the ECALLs served by the oracle's restatement of
the enclave (tests only).  The GPU test runs the same round trip on the HIP enclave.
"""
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, gpu_available

grpc = pytest.importorskip("grpc")

from fltee import wire  # noqa: E402


@pytest.fixture(scope="module")
def fx():
    return np.load(os.path.join(GOLDEN, "wire.npz"))


def _start_req(fx):
    return dict(fl_id=0, client_ids=list(range(100)), sigma=float(fx["start_sigma"]),
                clipping=float(fx["start_clipping"]), alpha=float(fx["start_alpha"]),
                sampling_ratio=float(fx["start_ratio"]), aggregation_alg=1,
                num_of_parameters=int(fx["d"]), num_of_sparse_parameters=int(fx["k"]))


def _agg_req(fx):
    return dict(fl_id=0, round=0, encrypted_parameters=fx["ciphertext"].tobytes(),
                num_of_parameters=int(fx["d"]), num_of_sparse_parameters=int(fx["k"]),
                optimal_num_of_clients=100, aggregation_alg=1,
                client_ids=[int(x) for x in fx["client_ids"]])


def test_encoding_is_byte_identical_to_reference_pb2(fx):
    ids = [int(x) for x in fx["client_ids"]]
    assert wire.encode_start_request(_start_req(fx)) == fx["start_req"].tobytes()
    assert wire.encode_start_response(dict(fl_id=0, round=0, client_ids=ids)) == fx["start_resp"].tobytes()
    assert wire.encode_aggregate_request(_agg_req(fx)) == fx["agg_req"].tobytes()
    resp = dict(updated_parameters=fx["updated"], execution_time=0.125, client_ids=ids[::-1], round=1)
    assert wire.encode_aggregate_response(resp) == fx["agg_resp"].tobytes()
    edge = dict(fl_id=4294967295, round=70000, client_ids=[int(x) for x in fx["edge_ids"]])
    assert wire.encode_start_response(edge) == fx["start_resp_edge"].tobytes()
    assert wire.encode_aggregate_request({}) == b"" == fx["agg_req_empty"].tobytes()


def test_decoding_reference_messages(fx):
    r = wire.decode_start_request(fx["start_req"].tobytes())
    assert r["client_ids"] == list(range(100)) and r["num_of_parameters"] == int(fx["d"])
    assert np.float32(r["sigma"]) == fx["start_sigma"] and np.float32(r["sampling_ratio"]) == fx["start_ratio"]
    a = wire.decode_aggregate_request(fx["agg_req"].tobytes())
    assert bytes(a["encrypted_parameters"]) == fx["ciphertext"].tobytes()
    assert a["client_ids"] == [int(x) for x in fx["client_ids"]] and a["optimal_num_of_clients"] == 100
    o = wire.decode_aggregate_response(fx["agg_resp"].tobytes())
    assert np.array_equal(o["updated_parameters"].view(np.uint32), fx["updated"].view(np.uint32))
    assert o["round"] == 1 and np.float32(o["execution_time"]) == np.float32(0.125)
    e = wire.decode_start_response(fx["start_resp_edge"].tobytes())
    assert e["client_ids"] == [int(x) for x in fx["edge_ids"]] and e["fl_id"] == 4294967295
    z = wire.decode_aggregate_request(b"")
    assert z["fl_id"] == 0 and len(z["encrypted_parameters"]) == 0 and z["client_ids"] == []


def test_decoder_accepts_unpacked_repeated_and_skips_unknown_fields():
    # client_ids (8) as three unpacked varints, an unknown fixed64 (15) and an unknown
    # length-delimited (16) field, updated_parameters-style unpacked floats in a response
    msg = (bytes([8 << 3 | 0, 5, 8 << 3 | 0, 0xAC, 0x02, 8 << 3 | 0, 7])
           + bytes([15 << 3 | 1]) + b"\x00" * 8 + wire._key(16, wire.LEN) + bytes([2]) + b"zz"
           + bytes([1 << 3 | 0, 9]))
    r = wire.decode_aggregate_request(msg)
    assert r["client_ids"] == [5, 300, 7] and r["fl_id"] == 9
    resp = (bytes([1 << 3 | 5]) + struct.pack("<f", 1.5) + bytes([1 << 3 | 5]) + struct.pack("<f", -2.0))
    assert wire.decode_aggregate_response(resp)["updated_parameters"].tolist() == [1.5, -2.0]
    with pytest.raises(wire.DecodeError):
        wire.decode_aggregate_request(bytes([3 << 3 | 2, 10, 1, 2]))  # truncated bytes field


class _OracleBackedEnclave:
    """fltee.ecalls.Enclave's method surface over the oracle's ECALL restatement
    (CPU tests only — the product path has no CPU fallback)."""

    def __init__(self, oracle):
        self.e = oracle.OracleEnclave(seed=99)

    def ecall_fl_init(self, fl_id, ids, d, k, sigma, clipping, alpha, ratio, alg, verbose, dp):
        return 0, self.e.fl_init(fl_id, ids, d, k, sigma, clipping, alpha, ratio, alg, verbose, dp)

    def ecall_start_round(self, fl_id, rnd, sample_size):
        rv, out = self.e.start_round(fl_id, rnd, sample_size)
        return 0, rv, out

    def ecall_secure_aggregation(self, fl_id, rnd, ids, enc, d, k, alg):
        rv, out, times = self.e.secure_aggregation(fl_id, rnd, ids, enc, d, k, alg)
        return 0, rv, out, times

    def ecall_client_size_optimized_secure_aggregation(self, fl_id, rnd, b, ids, enc, d, k, alg):
        rv, out, times = self.e.client_size_optimized_secure_aggregation(fl_id, rnd, b, ids, enc, d, k, alg)
        return 0, rv, out, times


def _round_trip(enclave, fx, alg):
    from fltee.grpc_server import Client, make_server
    from fltee.server import Aggregator
    server, port = make_server(Aggregator(enclave=enclave), "127.0.0.1:0", verbose=False)
    server.start()
    try:
        c = Client(f"127.0.0.1:{port}")
        ids = [int(x) for x in fx["client_ids"]]
        s = c.Start(fl_id=0, client_ids=ids, sigma=1.12, clipping=1.0, alpha=0.1, sampling_ratio=1.0,
                    aggregation_alg=alg, num_of_parameters=int(fx["d"]),
                    num_of_sparse_parameters=int(fx["k"]))
        assert s["round"] == 0 and sorted(s["client_ids"]) == sorted(ids)
        req = _agg_req(fx)
        req["aggregation_alg"] = alg
        r = c.Aggregate(**req)
        assert r["round"] == 1 and sorted(r["client_ids"]) == sorted(ids)
        # a replay of round 0 is refused by the enclave's state machine -> server panic
        with pytest.raises(grpc.RpcError) as ei:
            c.Aggregate(**req)
        assert ei.value.code() == grpc.StatusCode.INTERNAL
        c.close()
        return r["updated_parameters"]
    finally:
        server.stop(0)


def test_grpc_round_trip_oracle_enclave(fx, oracle):
    out = _round_trip(_OracleBackedEnclave(oracle), fx, alg=1)
    assert np.array_equal(out.view(np.uint32), fx["updated"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("alg", [1, 4])
def test_grpc_round_trip_gpu_enclave(fx, oracle, alg):
    from fltee.ecalls import Enclave
    out = _round_trip(Enclave(0), fx, alg=alg)
    w = oracle.decrypt_and_parse(fx["client_ids"], fx["ciphertext"])
    n, d, k = len(fx["client_ids"]), int(fx["d"]), int(fx["k"])
    ref = oracle.advanced(k, w, d, n)[0] if alg == 1 else oracle.non_oblivious(w, d, n)[0]
    assert np.array_equal(out.view(np.uint32), np.asarray(ref, np.float32).view(np.uint32))

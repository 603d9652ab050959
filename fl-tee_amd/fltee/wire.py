"""proto/secure_aggregation.proto on the wire, without generated code.

The four messages of the `secure_aggregation.Aggregator` service (proto:1-41) are
flat proto3 messages of uint32 / float / bytes scalars and packed repeated uint32 /
float fields, so a ~100-line codec serves them exactly:

  * encoding follows proto3 / the reference's Python pb2 byte for byte: fields in
    field-number order, scalars at their default value omitted, repeated scalars
    packed (tests/test_wire.py checks this against fixtures encoded by the
    reference's own secure_aggregation_pb2);
  * decoding accepts packed and unpacked repeated fields and skips unknown
    fields, like any proto3 parser;
  * `encrypted_parameters` (up to ~1 GB) is returned as a zero-copy memoryview
    slice of the request buffer and `updated_parameters` is (de)serialised with
    numpy, so the codec never loops in Python over the payload.
"""
import struct

import numpy as np

VARINT, I64, LEN, I32 = 0, 1, 2, 5

# field number -> (name, kind); kind: u32 | f32 | bytes | ru32 (repeated) | rf32 (repeated)
AGGREGATE_REQUEST = {1: ("fl_id", "u32"), 2: ("round", "u32"), 3: ("encrypted_parameters", "bytes"),
                     4: ("num_of_parameters", "u32"), 5: ("num_of_sparse_parameters", "u32"),
                     6: ("optimal_num_of_clients", "u32"), 7: ("aggregation_alg", "u32"),
                     8: ("client_ids", "ru32")}
AGGREGATE_RESPONSE = {1: ("updated_parameters", "rf32"), 2: ("execution_time", "f32"),
                      3: ("client_ids", "ru32"), 4: ("round", "u32")}
START_REQUEST = {1: ("fl_id", "u32"), 2: ("client_ids", "ru32"), 3: ("sigma", "f32"),
                 4: ("clipping", "f32"), 5: ("alpha", "f32"), 6: ("sampling_ratio", "f32"),
                 7: ("aggregation_alg", "u32"), 8: ("num_of_parameters", "u32"),
                 9: ("num_of_sparse_parameters", "u32")}
START_RESPONSE = {1: ("fl_id", "u32"), 2: ("round", "u32"), 3: ("client_ids", "ru32")}


class DecodeError(ValueError):
    pass


def _varint(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, i):
    shift = result = 0
    while True:
        if i >= len(buf):
            raise DecodeError("truncated varint")
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7
        if shift >= 64:
            raise DecodeError("varint too long")


def _key(num, wt):
    return _varint((num << 3) | wt)


def encode(schema, msg):
    """msg: dict of field name -> value (missing = default)."""
    out = []
    for num in sorted(schema):
        name, kind = schema[num]
        v = msg.get(name)
        if v is None:
            continue
        if kind == "u32":
            v = int(v) & 0xFFFFFFFF
            if v:
                out += [_key(num, VARINT), _varint(v)]
        elif kind == "f32":
            if float(v) != 0.0:  # prost (server.rs) and pure-Python pb2: == 0.0 is omitted
                out += [_key(num, I32), struct.pack("<f", float(v))]
        elif kind == "bytes":
            if len(v):
                out += [_key(num, LEN), _varint(len(v)), bytes(v)]
        elif kind == "ru32":
            a = np.asarray(v, dtype=np.uint64).reshape(-1)
            if a.size:
                body = b"".join(_varint(int(x) & 0xFFFFFFFF) for x in a)
                out += [_key(num, LEN), _varint(len(body)), body]
        elif kind == "rf32":
            a = np.ascontiguousarray(v, dtype="<f4").reshape(-1)
            if a.size:
                out += [_key(num, LEN), _varint(a.nbytes), a.tobytes()]
        else:
            raise ValueError(kind)
    return b"".join(out)


def decode(schema, data):
    buf = memoryview(data).cast("B") if not isinstance(data, memoryview) else data.cast("B")
    msg = {}
    for name, kind in schema.values():
        msg[name] = ([] if kind in ("ru32",) else
                     np.zeros(0, np.float32) if kind == "rf32" else
                     memoryview(b"") if kind == "bytes" else
                     0.0 if kind == "f32" else 0)
    i, n = 0, len(buf)
    while i < n:
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        field = schema.get(num)
        kind = field[1] if field else None
        if wt == VARINT:
            v, i = _read_varint(buf, i)
            if kind == "u32":
                msg[field[0]] = v & 0xFFFFFFFF
            elif kind == "ru32":
                msg[field[0]].append(v & 0xFFFFFFFF)
        elif wt == I32:
            if i + 4 > n:
                raise DecodeError("truncated fixed32")
            if kind == "f32":
                msg[field[0]] = struct.unpack_from("<f", buf, i)[0]
            elif kind == "rf32":
                msg[field[0]] = np.concatenate([msg[field[0]], np.frombuffer(buf[i:i + 4], "<f4")])
            i += 4
        elif wt == I64:
            i += 8
        elif wt == LEN:
            ln, i = _read_varint(buf, i)
            if i + ln > n:
                raise DecodeError("truncated length-delimited field")
            body = buf[i:i + ln]
            i += ln
            if kind == "bytes":
                msg[field[0]] = body
            elif kind == "ru32":
                j = 0
                while j < ln:
                    v, j = _read_varint(body, j)
                    msg[field[0]].append(v & 0xFFFFFFFF)
            elif kind == "rf32":
                if ln % 4:
                    raise DecodeError("packed float field of odd length")
                msg[field[0]] = np.concatenate([msg[field[0]], np.frombuffer(body, "<f4")])
        else:
            raise DecodeError(f"unsupported wire type {wt}")
    if i != n:
        raise DecodeError("trailing bytes")
    return msg


def decode_aggregate_request(b):
    return decode(AGGREGATE_REQUEST, b)


def encode_aggregate_request(m):
    return encode(AGGREGATE_REQUEST, m)


def decode_aggregate_response(b):
    return decode(AGGREGATE_RESPONSE, b)


def encode_aggregate_response(m):
    return encode(AGGREGATE_RESPONSE, m)


def decode_start_request(b):
    return decode(START_REQUEST, b)


def encode_start_request(m):
    return encode(START_REQUEST, m)


def decode_start_response(b):
    return decode(START_RESPONSE, b)


def encode_start_response(m):
    return encode(START_RESPONSE, m)

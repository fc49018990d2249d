"""Minimal protobuf wire-format encoder/decoder for the few TF protos the framework writes:
Event/Summary (TensorBoard event files), TrackableObjectGraph (tf.train.Checkpoint),
CheckpointState is text format (see train/checkpoint.py).

Field encoders take python values; messages are plain bytes. Decoding returns a dict
field_number -> list of raw values (ints for varint/fixed, bytes for length-delimited).
"""
from __future__ import annotations

import struct
from typing import Dict, List


def varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def tag(field: int, wire: int) -> bytes:
    return varint((field << 3) | wire)


def f_varint(field: int, v: int, keep_zero=False) -> bytes:
    if v == 0 and not keep_zero:
        return b""
    return tag(field, 0) + varint(int(v))


def f_bool(field: int, v: bool) -> bytes:
    return f_varint(field, 1 if v else 0)


def f_double(field: int, v: float) -> bytes:
    return tag(field, 1) + struct.pack("<d", v)


def f_float(field: int, v: float) -> bytes:
    return tag(field, 5) + struct.pack("<f", v)


def f_fixed32(field: int, v: int) -> bytes:
    return tag(field, 5) + struct.pack("<I", v)


def f_bytes(field: int, b: bytes) -> bytes:
    return tag(field, 2) + varint(len(b)) + b


def f_str(field: int, s: str) -> bytes:
    return f_bytes(field, s.encode("utf-8"))


def f_msg(field: int, b: bytes) -> bytes:
    return f_bytes(field, b)


def _read_varint(buf: bytes, i: int):
    r, shift = 0, 0
    while True:
        b = buf[i]
        i += 1
        r |= (b & 0x7F) << shift
        if not b & 0x80:
            return r, i
        shift += 7


def decode(buf: bytes) -> Dict[int, List]:
    out: Dict[int, List] = {}
    i = 0
    while i < len(buf):
        t, i = _read_varint(buf, i)
        field, wire = t >> 3, t & 7
        if wire == 0:
            v, i = _read_varint(buf, i)
        elif wire == 1:
            v = struct.unpack_from("<Q", buf, i)[0]
            i += 8
        elif wire == 2:
            n, i = _read_varint(buf, i)
            v = bytes(buf[i:i + n])
            i += n
        elif wire == 5:
            v = struct.unpack_from("<I", buf, i)[0]
            i += 4
        else:
            raise ValueError("unsupported wire type %d" % wire)
        out.setdefault(field, []).append(v)
    return out


def as_double(v: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", v))[0]


def as_float(v: int) -> float:
    return struct.unpack("<f", struct.pack("<I", v))[0]

"""TensorBoard event files, written through the native TFRecord writer
(csrc/runtime/record_io.cc, masked-crc32c framing).

Reference: the `loss_<task>` / `accuracy_<task>` scalar summaries
(/root/reference/distribute_training.py:128-132) written every 100 steps by
MonitoredTrainingSession's chief-only SummarySaverHook, plus StepCounterHook's
`global_step/sec`.

  Event   { double wall_time = 1; int64 step = 2; string file_version = 3; Summary summary = 5; }
  Summary { repeated Value value = 1; }   Value { string tag = 1; float simple_value = 2; }
"""
from __future__ import annotations

import ctypes
import os
import socket
import threading
import time
from typing import Iterator, List, Optional, Tuple

from .. import _native
from . import proto


def _rt():
    lib = _native.rt()
    if not getattr(lib, "_rec_sigs", False):
        lib.ttd_record_writer_open.restype = ctypes.c_void_p
        lib.ttd_record_writer_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
        lib.ttd_record_writer_write.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64]
        lib.ttd_record_writer_flush.argtypes = [ctypes.c_void_p]
        lib.ttd_record_writer_close.argtypes = [ctypes.c_void_p]
        lib.ttd_record_reader_open.restype = ctypes.c_void_p
        lib.ttd_record_reader_open.argtypes = [ctypes.c_char_p]
        lib.ttd_record_reader_next.restype = ctypes.c_int64
        lib.ttd_record_reader_next.argtypes = [ctypes.c_void_p]
        lib.ttd_record_reader_data.restype = ctypes.c_void_p
        lib.ttd_record_reader_data.argtypes = [ctypes.c_void_p]
        lib.ttd_record_reader_close.argtypes = [ctypes.c_void_p]
        lib.ttd_crc32c_extend.restype = ctypes.c_uint32
        lib.ttd_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        lib.ttd_crc32c_mask.restype = ctypes.c_uint32
        lib.ttd_crc32c_mask.argtypes = [ctypes.c_uint32]
        lib._rec_sigs = True
    return lib


def crc32c(data: bytes) -> int:
    return _rt().ttd_crc32c_extend(0, data, len(data))


def masked_crc32c(data: bytes) -> int:
    lib = _rt()
    return lib.ttd_crc32c_mask(lib.ttd_crc32c_extend(0, data, len(data)))


class RecordWriter:
    def __init__(self, path: str, append: bool = False):
        self._h = _rt().ttd_record_writer_open(path.encode(), 1 if append else 0)
        if not self._h:
            raise IOError(_native.rt_error())
        self.path = path

    def write(self, data: bytes):
        if _rt().ttd_record_writer_write(self._h, data, len(data)) != 0:
            raise IOError(_native.rt_error())

    def flush(self):
        _rt().ttd_record_writer_flush(self._h)

    def close(self):
        if self._h:
            _rt().ttd_record_writer_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_records(path: str) -> Iterator[bytes]:
    lib = _rt()
    h = lib.ttd_record_reader_open(path.encode())
    if not h:
        raise IOError(_native.rt_error())
    try:
        while True:
            n = lib.ttd_record_reader_next(h)
            if n == -1:
                return
            if n < 0:
                raise IOError("corrupt record in %s: %s" % (path, _native.rt_error()))
            yield ctypes.string_at(lib.ttd_record_reader_data(h), n)
    finally:
        lib.ttd_record_reader_close(h)


# ------------------------------------------------------------------ Event / Summary protos
def summary_value_scalar(tag: str, value: float) -> bytes:
    return proto.f_str(1, tag) + proto.f_float(2, float(value))


def summary_proto(values: List[bytes]) -> bytes:
    return b"".join(proto.f_msg(1, v) for v in values)


def event_proto(wall_time: float, step: int = 0, summary: Optional[bytes] = None,
                file_version: Optional[str] = None) -> bytes:
    out = proto.f_double(1, wall_time) + proto.f_varint(2, step)
    if file_version is not None:
        out += proto.f_str(3, file_version)
    if summary is not None:
        out += proto.f_msg(5, summary)
    return out


def parse_event(buf: bytes) -> dict:
    d = proto.decode(buf)
    ev = {"wall_time": proto.as_double(d[1][0]) if 1 in d else 0.0, "step": d.get(2, [0])[0]}
    if 3 in d:
        ev["file_version"] = d[3][0].decode()
    if 5 in d:
        vals = []
        for v in proto.decode(d[5][0]).get(1, []):
            vd = proto.decode(v)
            vals.append((vd[1][0].decode(), proto.as_float(vd[2][0]) if 2 in vd else None))
        ev["summary"] = vals
    return ev


class EventFileWriter:
    """Appends Events to `<logdir>/events.out.tfevents.<unix ts>.<host>` from a background
    thread (non-blocking add_event, periodic flush)."""

    def __init__(self, logdir: str, flush_secs: float = 120.0, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        self.path = os.path.join(logdir, "events.out.tfevents.%010d.%s%s"
                                 % (int(time.time()), socket.gethostname(), filename_suffix))
        self._w = RecordWriter(self.path)
        self._lock = threading.Lock()
        self._w.write(event_proto(time.time(), 0, file_version="brain.Event:2"))
        self._w.flush()
        self._flush_secs = flush_secs
        self._last_flush = time.time()
        self._closed = False

    def add_event(self, ev: bytes):
        with self._lock:
            if self._closed:
                return
            self._w.write(ev)
            if time.time() - self._last_flush > self._flush_secs:
                self._w.flush()
                self._last_flush = time.time()

    def add_summary(self, summary: bytes, global_step: int = 0):
        self.add_event(event_proto(time.time(), int(global_step), summary=summary))

    def add_scalars(self, scalars, global_step: int):
        self.add_summary(summary_proto([summary_value_scalar(t, v) for t, v in scalars]), global_step)

    def flush(self):
        with self._lock:
            if not self._closed:
                self._w.flush()

    def close(self):
        with self._lock:
            if not self._closed:
                self._w.flush()
                self._w.close()
                self._closed = True


def read_events(path: str) -> List[dict]:
    return [parse_event(r) for r in read_records(path)]

"""Minimal TensorBoard event-file writer (``tensorboard`` is not installed here).

Replaces ``torch.utils.tensorboard.SummaryWriter`` used by the reference trainer
(``modules/model/trainer/trainer.py:183-192,215-219``) for scalar summaries only.
File format = TFRecord framing around hand-encoded ``Event`` protobufs:

    uint64 length | uint32 masked_crc32c(length) | bytes event | uint32 masked_crc32c(event)

``Event{1: wall_time (double), 2: step (int64), 3: file_version (string) | 5: Summary}``,
``Summary{1: repeated Value}``, ``Value{1: tag (string), 2: simple_value (float)}``.
The CRC32C (Castagnoli) runs in the native host library when it is built, else in Python.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Optional

_CRC_TABLE = None


def _crc32c_py(data: bytes) -> int:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        table = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            table.append(c)
        _CRC_TABLE = table
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def crc32c(data: bytes) -> int:
    try:
        from .._native import host
        return host().crc32c(data)
    except Exception:  # host lib not built yet: pure-python path (TB writing is off the hot path)
        return _crc32c_py(data)


def masked_crc32c(data: bytes) -> int:
    crc = crc32c(data)
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, *, file_version: Optional[str] = None, scalars=None) -> bytes:
    ev = _varint((1 << 3) | 1) + struct.pack("<d", wall_time)
    ev += _varint((2 << 3) | 0) + _varint(int(step))
    if file_version is not None:
        ev += _field_bytes(3, file_version.encode())
    if scalars:
        summary = b""
        for tag, value in scalars:
            val = _field_bytes(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(value))
            summary += _field_bytes(1, val)
        ev += _field_bytes(5, summary)
    return ev


def frame_record(data: bytes) -> bytes:
    header = struct.pack("<Q", len(data))
    return header + struct.pack("<I", masked_crc32c(header)) + data + struct.pack("<I", masked_crc32c(data))


class SummaryWriter:
    """Scalar-only drop-in for ``torch.utils.tensorboard.SummaryWriter``."""

    def __init__(self, log_dir: str, flush_secs: float = 10.0):
        self.log_dir = str(log_dir)
        os.makedirs(self.log_dir, exist_ok=True)
        fname = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.0"
        self.path = os.path.join(self.log_dir, fname)
        self._f = open(self.path, "wb")
        self._f.write(frame_record(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self._flush_secs = flush_secs
        self._last_flush = time.time()

    def add_scalar(self, tag: str, scalar_value, global_step: int = 0, walltime: Optional[float] = None):
        if hasattr(scalar_value, "item"):
            scalar_value = scalar_value.item()
        ev = encode_event(walltime or time.time(), global_step, scalars=[(tag, scalar_value)])
        self._f.write(frame_record(ev))
        if time.time() - self._last_flush > self._flush_secs:
            self.flush()

    def add_scalars_batch(self, scalars, global_step: int):
        ev = encode_event(time.time(), global_step, scalars=list(scalars))
        self._f.write(frame_record(ev))

    def flush(self):
        self._f.flush()
        self._last_flush = time.time()

    def close(self):
        if not self._f.closed:
            self._f.flush()
            self._f.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_events(path: str):
    """Parse an event file back into ``[(step, tag, value)]`` (used by tests / tooling)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        (length,) = struct.unpack_from("<Q", data, pos)
        (hcrc,) = struct.unpack_from("<I", data, pos + 8)
        assert hcrc == masked_crc32c(data[pos:pos + 8]), "header crc mismatch"
        ev = data[pos + 12:pos + 12 + length]
        (dcrc,) = struct.unpack_from("<I", data, pos + 12 + length)
        assert dcrc == masked_crc32c(ev), "data crc mismatch"
        pos += 16 + length
        out.extend(_decode_event(ev))
    return out


def _read_varint(buf, i):
    shift = 0
    result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def _iter_fields(buf):
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        else:
            raise ValueError(f"wire type {wt}")
        yield num, wt, v


def _decode_event(ev):
    step = 0
    out = []
    for num, wt, v in _iter_fields(ev):
        if num == 2:
            step = v
        elif num == 5:
            for n2, _, val in _iter_fields(v):
                if n2 != 1:
                    continue
                tag, value = None, None
                for n3, _, x in _iter_fields(val):
                    if n3 == 1:
                        tag = bytes(x).decode()
                    elif n3 == 2:
                        value = struct.unpack("<f", x)[0]
                out.append((tag, value))
    return [(step, t, v) for t, v in out]

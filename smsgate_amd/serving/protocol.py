"""Binary wire format between parser processes and a GPU engine server.

Requests and responses are token-id batches, packed with numpy (no pickle):

``request``  = ``b"Q"`` | req_id:u64 | n:u32 | lens:u16[n] | ids:i32[sum(lens)]
``response`` = ``b"R"`` | req_id:u64 | n:u32 | lens:u16[n] | ids:i32[sum(lens)]
``error``    = ``b"E"`` | req_id:u64 | utf-8 message
``control``  = ``b"C"`` | utf-8 JSON (used by the benchmark harness)

Tokenisation and detokenisation happen on the client side, so the GPU
process does only scheduling: its Python work per message is a few slices.
"""
from __future__ import annotations

import itertools
import json
import struct
from dataclasses import dataclass
from typing import Any, List, Sequence, Tuple

import numpy as np

__all__ = ["pack_ids", "pack_raw", "unpack_ids", "unpack_id_arrays", "unpack_arrays", "PackedAnswer", "pack_error", "pack_control", "kind", "req_id",
           "count", "HEADER_SIZE"]

_HDR = struct.Struct("<cQI")


def pack_ids(tag: bytes, req_id: int, seqs: Sequence[Sequence[int]]) -> bytes:
    n = len(seqs)
    lens = np.fromiter(map(len, seqs), dtype=np.uint16, count=n)
    flat = np.array(list(itertools.chain.from_iterable(seqs)), dtype=np.int32)
    return _HDR.pack(tag, req_id, n) + lens.tobytes() + flat.tobytes()


HEADER_SIZE = _HDR.size


def pack_raw(tag: bytes, req_id: int, n: int, lens: bytes, flat: bytes) -> bytes:
    """A frame from already-packed uint16 lengths and int32 ids (the native encoder's output)."""
    return _HDR.pack(tag, req_id, n) + lens + flat


def req_id(buf: bytes) -> int:
    return _HDR.unpack_from(buf, 0)[1]


def count(buf: bytes) -> int:
    return _HDR.unpack_from(buf, 0)[2]


def pack_arrays(tag: bytes, req_id: int, lens: np.ndarray, flat: np.ndarray) -> bytes:
    return _HDR.pack(tag, req_id, len(lens)) + lens.astype(np.uint16).tobytes() + flat.astype(np.int32).tobytes()


def unpack_ids(buf: bytes) -> Tuple[bytes, int, List[List[int]]]:
    tag, req_id, n = _HDR.unpack_from(buf, 0)
    off = _HDR.size
    lens = np.frombuffer(buf, dtype=np.uint16, count=n, offset=off)
    off += 2 * n
    flat = np.frombuffer(buf, dtype=np.int32, count=int(lens.sum()), offset=off).tolist()
    out: List[List[int]] = []
    p = 0
    for ln in lens.tolist():
        out.append(flat[p:p + ln])
        p += ln
    return tag, req_id, out


def unpack_id_arrays(buf: bytes) -> Tuple[bytes, int, List[np.ndarray]]:
    """As :func:`unpack_ids`, but each sequence is an int32 view into one copy of the
    payload (the engine server's path: no per-token Python objects)."""
    tag, req_id, n = _HDR.unpack_from(buf, 0)
    off = _HDR.size
    lens = np.frombuffer(buf, dtype=np.uint16, count=n, offset=off)
    off += 2 * n
    flat = np.frombuffer(buf, dtype=np.int32, count=int(lens.sum()), offset=off).copy()
    # plain slices (views of the one copy): np.split costs ~3 us per piece (array_split +
    # swapaxes per sub-array) on the GPU feeder's loop
    ends = np.cumsum(lens, dtype=np.int64).tolist()
    return tag, req_id, [flat[a:b] for a, b in zip([0] + ends[:-1], ends)]


@dataclass
class PackedAnswer:
    """Answers of a whole request (an engine's ``submit_packed`` unit): copy-format token
    lengths (uint16 [n]) and the ids back to back (int32) -- a response frame's arrays."""
    lens: np.ndarray
    flat: np.ndarray


def unpack_arrays(buf: bytes) -> Tuple[bytes, int, np.ndarray, np.ndarray]:
    """``(tag, req_id, lens int32 [n], ids int32 [sum(lens)])``: a frame as two arrays
    (a copy of the ids; the engine's packed-request path)."""
    tag, req_id, n = _HDR.unpack_from(buf, 0)
    off = _HDR.size
    lens = np.frombuffer(buf, dtype=np.uint16, count=n, offset=off).astype(np.int32)
    off += 2 * n
    flat = np.frombuffer(buf, dtype=np.int32, count=int(lens.sum()), offset=off).copy()
    return tag, req_id, lens, flat


def pack_error(req_id: int, msg: str) -> bytes:
    return _HDR.pack(b"E", req_id, 0) + msg.encode()


def unpack_error(buf: bytes) -> Tuple[int, str]:
    _, req_id, _ = _HDR.unpack_from(buf, 0)
    return req_id, buf[_HDR.size:].decode(errors="replace")


def pack_control(obj: Any) -> bytes:
    return b"C" + json.dumps(obj).encode()


def unpack_control(buf: bytes) -> Any:
    return json.loads(buf[1:].decode())


def kind(buf: bytes) -> bytes:
    return buf[:1]

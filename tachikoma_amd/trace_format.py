"""The tachikoma trace binary: writer (through the C ABI) and a numpy reader.

Container (``include/tachikoma.h``, "trace format")::

    tk_trace_header  {"TKTRACE\\0", version, json_len, params_off, params_size,
                      records_off, records_size}       (7 × u64, little-endian)
    json             op table + run metadata (utf-8, space padded)
    pad to 4096
    params blob      NDArray-list (src/runtime/file_utils.cc:210-236) of the weights
    pad to 4096
    records blob     NDArray-list of every traced tensor: graph inputs, then every
                     op output in topological order, keyed by MRT symbol name (%N)

Each record is the whole batch shard of that op output ([B_shard, ...]), i.e.
exactly what ``mrt.Trace.calibrate`` returns per symbol
(python/tvm/mrt/trace.py:65-117); ``sample_offset`` in the json places the shard
in the global batch.  The NDArray-list encoding makes the params/records
sections loadable by the reference's own ``LoadParams`` / CRT reader.
"""
from __future__ import annotations

import ctypes
import json
import mmap
import os
import struct
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

TRACE_MAGIC = 0x0045434152544B54
TRACE_VERSION = 1
TRACE_ALIGN = 4096
LIST_MAGIC = 0xF7E58D4F05049CB7
ARRAY_MAGIC = 0xDD5E40F096B4A13F
JSON_SLACK = 256  # header json is space-padded so per-shard fields can be rewritten in place


def _metas(items: Sequence[Tuple[str, Sequence[int], str]]):
    """Build a ctypes tk_array_meta array (+ keepalive list)."""
    keep = []
    arr = (_lib.tk_array_meta * max(1, len(items)))()
    for i, (name, shape, dtype) in enumerate(items):
        nm = name.encode()
        sh = (ctypes.c_int64 * max(1, len(shape)))(*[int(s) for s in shape])
        keep += [nm, sh]
        arr[i].name = nm
        arr[i].ndim = len(shape)
        arr[i].shape = ctypes.cast(sh, ctypes.POINTER(ctypes.c_int64))
        arr[i].dtype = _lib.dtype_struct(dtype)
    return arr, keep


@dataclass
class TraceLayout:
    json_text: str
    total: int
    param_offsets: List[int]
    record_offsets: List[int]
    params: List[Tuple[str, Tuple[int, ...], str]]
    records: List[Tuple[str, Tuple[int, ...], str]]

    @staticmethod
    def compute(json_text: str, params, records) -> "TraceLayout":
        lib = _lib.load()
        pm, k1 = _metas(params)
        rm, k2 = _metas(records)
        po = (ctypes.c_int64 * max(1, len(params)))()
        ro = (ctypes.c_int64 * max(1, len(records)))()
        total = lib.tk_trace_layout(json_text.encode(), pm, len(params), rm, len(records), po, ro)
        if total < 0:
            _lib.check(int(total), "tk_trace_layout")
        return TraceLayout(json_text, int(total), list(po[:len(params)]), list(ro[:len(records)]),
                           list(params), list(records))

    def write_headers(self, image_ptr: int, image_size: int) -> None:
        lib = _lib.load()
        pm, k1 = _metas(self.params)
        rm, k2 = _metas(self.records)
        _lib.check(lib.tk_trace_write_headers(self.json_text.encode(), pm, len(self.params), rm, len(self.records),
                                              ctypes.c_void_p(image_ptr), image_size), "tk_trace_write_headers")


def save_ndarray_list(arrays: Dict[str, np.ndarray]) -> bytes:
    """NDArray-list blob (``SaveParams``, src/runtime/file_utils.cc:210-236) of host arrays, in
    insertion order, written through the C ABI (tk_ndlist_layout / tk_ndlist_write_headers)."""
    lib = _lib.load()
    items = [(k, tuple(np.asarray(v).shape), str(np.asarray(v).dtype)) for k, v in arrays.items()]
    metas, keep = _metas(items)
    offs = (ctypes.c_int64 * max(1, len(items)))()
    total = lib.tk_ndlist_layout(metas, len(items), offs)
    if total < 0:
        _lib.check(int(total), "tk_ndlist_layout")
    blob = bytearray(int(total))
    buf = (ctypes.c_char * len(blob)).from_buffer(blob)
    _lib.check(lib.tk_ndlist_write_headers(metas, len(items), buf, len(blob)), "tk_ndlist_write_headers")
    for i, v in enumerate(arrays.values()):
        raw = np.ascontiguousarray(v).reshape(-1).view(np.uint8)
        blob[offs[i]:offs[i] + raw.size] = raw.tobytes()
    return bytes(blob)


def header_json(meta: Dict[str, Any]) -> str:
    text = json.dumps(meta, separators=(",", ":"), sort_keys=False)
    return text + " " * JSON_SLACK


def write_file(path: str, image_ptr: int, size: int) -> None:
    _lib.check(_lib.load().tk_write_file(path.encode(), ctypes.c_void_p(image_ptr), size), "tk_write_file")


# ---------------------------------------------------------------- numpy reader

def _np_dtype(code: int, bits: int) -> np.dtype:
    kind = {0: "i", 1: "u", 2: "f"}[code]
    return np.dtype(f"<{kind}{bits // 8}")


def parse_ndarray_list(buf, offset: int = 0, size: Optional[int] = None, copy: bool = False) -> Dict[str, np.ndarray]:
    """Parse an NDArray-list blob (LoadParams, src/runtime/file_utils.cc:184-206)."""
    mv = memoryview(buf)
    end = len(mv) if size is None else offset + size
    off = offset

    def rd(fmt):
        nonlocal off
        n = struct.calcsize(fmt)
        if off + n > end:
            raise ValueError("truncated NDArray-list blob")
        v = struct.unpack_from(fmt, mv, off)
        off += n
        return v

    magic, _ = rd("<QQ")
    if magic != LIST_MAGIC:
        raise ValueError("not an NDArray-list blob")
    (n,) = rd("<Q")
    names = []
    for _ in range(n):
        (ln,) = rd("<Q")
        names.append(bytes(mv[off:off + ln]).decode())
        off += ln
    (na,) = rd("<Q")
    if na != n:
        raise ValueError("name/array count mismatch")
    out: Dict[str, np.ndarray] = {}
    for name in names:
        amagic, _, dev_type, dev_id, ndim = rd("<QQiii")
        if amagic != ARRAY_MAGIC:
            raise ValueError("bad array magic")
        code, bits, lanes = rd("<BBH")
        shape = rd(f"<{ndim}q") if ndim else ()
        (nbytes,) = rd("<q")
        dt = _np_dtype(code, bits)
        arr = np.frombuffer(mv, dtype=dt, count=nbytes // dt.itemsize, offset=off).reshape(shape)
        out[name] = arr.copy() if copy else arr
        off += nbytes
    return out


@dataclass
class Trace:
    meta: Dict[str, Any]
    params: Dict[str, np.ndarray]
    records: Dict[str, np.ndarray]


def read_trace(path_or_bytes, copy: bool = False) -> Trace:
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
        buf = path_or_bytes
    else:
        with open(path_or_bytes, "rb") as f:
            buf = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    magic, version, jl, po, ps, ro, rs = struct.unpack_from("<7Q", buf, 0)
    if magic != TRACE_MAGIC:
        raise ValueError("not a tachikoma trace (bad magic)")
    if version != TRACE_VERSION:
        raise ValueError(f"unsupported trace version {version}")
    meta = json.loads(bytes(buf[56:56 + jl]).decode())
    params = parse_ndarray_list(buf, po, ps, copy=copy)
    records = parse_ndarray_list(buf, ro, rs, copy=copy)
    return Trace(meta, params, records)


# ---------------------------------------------------------------- digests
# Host twin of the device digest (tk_digest_bytes, csrc/tk_elementwise.hip):
#   D(bytes) = Σ_i splitmix64_final(w_i ^ i·0x9E3779B97F4A7C15)  mod 2^64
# over little-endian 8-byte words w_i, the tail zero-padded.  The trace digest of a
# shard is D over the u64 array [D(record_0), D(record_1), ...] in record order, so
# it can be recomputed from a trace file without the GPU.

_PHI = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def digest_bytes(buf, chunk_words: int = 1 << 22) -> int:
    raw = np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8)
    nw = (raw.size + 7) // 8
    total = np.uint64(0)
    full = raw.size // 8
    with np.errstate(over="ignore"):
        for s in range(0, nw, chunk_words):
            e = min(nw, s + chunk_words)
            if e <= full:
                w = raw[s * 8:e * 8].view("<u8")
            else:
                tail = np.zeros((e - s) * 8, np.uint8)
                part = raw[s * 8:]
                tail[:part.size] = part
                w = tail.view("<u8")
            idx = np.arange(s, e, dtype=np.uint64)
            total = total + np.sum(_mix64(w ^ (idx * _PHI)), dtype=np.uint64)
    return int(total)


def records_digest(records: "Dict[str, np.ndarray] | Sequence[np.ndarray]") -> int:
    """Digest of a shard's records in trace order (graph inputs first, then ops)."""
    arrays = list(records.values()) if isinstance(records, dict) else list(records)
    per = np.array([digest_bytes(np.ascontiguousarray(a).reshape(-1).view(np.uint8)) for a in arrays],
                   dtype=np.uint64)
    return digest_bytes(per.tobytes())


def trace_file_digest(path_or_bytes) -> int:
    return records_digest(read_trace(path_or_bytes).records)


def trace_bytes(meta: Dict[str, Any], params: Dict[str, np.ndarray], records: Dict[str, np.ndarray]) -> bytes:
    """A complete trace file from host arrays (the same layout the device capture fills:
    tk_trace_layout / tk_trace_write_headers), e.g. for traces produced on the CPU."""
    p_items = [(k, tuple(np.asarray(v).shape), str(np.asarray(v).dtype)) for k, v in params.items()]
    r_items = [(k, tuple(np.asarray(v).shape), str(np.asarray(v).dtype)) for k, v in records.items()]
    layout = TraceLayout.compute(header_json(meta), p_items, r_items)
    blob = bytearray(layout.total)
    buf = (ctypes.c_char * len(blob)).from_buffer(blob)
    layout.write_headers(ctypes.addressof(buf), len(blob))
    del buf
    for offs, arrays in ((layout.param_offsets, params.values()), (layout.record_offsets, records.values())):
        for off, v in zip(offs, arrays):
            raw = np.ascontiguousarray(v).reshape(-1).view(np.uint8)
            blob[off:off + raw.size] = raw.tobytes()
    return bytes(blob)

"""Restatement of the reference's NDArray-list encoding (TEST INFRASTRUCTURE ONLY).

Writer: SaveParams (src/runtime/file_utils.cc:210-236) + SaveDLTensor
(include/tvm/runtime/ndarray.h:449-494), with dmlc::Stream's vector<string>
encoding (u64 count, then u64 length + bytes per name).  Reader: LoadParams
(file_utils.cc:184-206) / TVMNDArray_Load (src/runtime/crt/common/ndarray.c:72-131).
Independent of tachikoma_amd's C++ writer, so the two cross-check each other.
"""
import struct

import numpy as np

LIST_MAGIC = 0xF7E58D4F05049CB7
ARRAY_MAGIC = 0xDD5E40F096B4A13F
_CODES = {"i": 0, "u": 1, "f": 2}


def save_params(arrays):
    """arrays: list of (name, np.ndarray) in the order to write."""
    out = [struct.pack("<QQ", LIST_MAGIC, 0), struct.pack("<Q", len(arrays))]
    for name, _ in arrays:
        b = name.encode()
        out.append(struct.pack("<Q", len(b)) + b)
    out.append(struct.pack("<Q", len(arrays)))
    for _, a in arrays:
        a = np.asarray(a).copy(order="C")  # (np.ascontiguousarray would promote rank 0 to rank 1)
        code = _CODES[a.dtype.kind]
        out.append(struct.pack("<QQ", ARRAY_MAGIC, 0))
        out.append(struct.pack("<ii", 1, 0))            # kDLCPU, device 0
        out.append(struct.pack("<i", a.ndim))
        out.append(struct.pack("<BBH", code, a.dtype.itemsize * 8, 1))
        out.append(struct.pack(f"<{a.ndim}q", *a.shape))
        out.append(struct.pack("<q", a.nbytes))
        out.append(a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes())
    return b"".join(out)


def load_params(blob):
    mv = memoryview(blob)
    off = 0

    def rd(fmt):
        nonlocal off
        v = struct.unpack_from(fmt, mv, off)
        off += struct.calcsize(fmt)
        return v

    magic, _ = rd("<QQ")
    assert magic == LIST_MAGIC, "Invalid parameters file format"
    (n,) = rd("<Q")
    names = []
    for _ in range(n):
        (ln,) = rd("<Q")
        names.append(bytes(mv[off:off + ln]).decode())
        off += ln
    (sz,) = rd("<Q")
    assert sz == n, "Invalid parameters file format"
    out = {}
    for name in names:
        magic, _ = rd("<QQ")
        assert magic == ARRAY_MAGIC, "Invalid DLTensor file format"
        dev_type, dev_id, ndim = rd("<iii")
        code, bits, lanes = rd("<BBH")
        shape = rd(f"<{ndim}q") if ndim else ()
        (nbytes,) = rd("<q")
        kind = {0: "i", 1: "u", 2: "f"}[code]
        dt = np.dtype(f"<{kind}{bits // 8}")
        out[name] = np.frombuffer(bytes(mv[off:off + nbytes]), dtype=dt).reshape(shape)
        off += nbytes
    return out

"""Trace binary: the product's C++ NDArray-list writer is byte-identical to the oracle's
restatement of SaveParams, and traces round-trip through both readers."""
import ctypes

import numpy as np

from oracle import ndarray_list
from tachikoma_amd import _lib
from tachikoma_amd import trace_format as tf


def _arrays():
    rng = np.random.default_rng(0)
    return [("data", rng.integers(-128, 128, size=(2, 3, 4, 5)).astype(np.int8)),
            ("%0", rng.integers(-2**31, 2**31, size=(2, 8, 4, 5), dtype=np.int64).astype(np.int32)),
            ("%1", rng.integers(0, 256, size=(7,)).astype(np.uint8)),
            ("scalar", np.array(5, dtype=np.int32)),
            ("empty", np.zeros((0, 3), dtype=np.int16)),
            ("conv1.weight", rng.integers(-128, 128, size=(4, 3, 3, 3)).astype(np.int8))]


def _write_blob(arrays):
    lib = _lib.load()
    metas, keep = tf._metas([(n, a.shape, str(a.dtype)) for n, a in arrays])
    offs = (ctypes.c_int64 * len(arrays))()
    size = lib.tk_ndlist_layout(metas, len(arrays), offs)
    buf = np.zeros(size, dtype=np.uint8)
    _lib.check(lib.tk_ndlist_write_headers(metas, len(arrays), ctypes.c_void_p(buf.ctypes.data), size))
    for (n, a), off in zip(arrays, offs):
        buf[off:off + a.nbytes] = np.frombuffer(a.tobytes(), dtype=np.uint8)
    return buf.tobytes()


def test_ndlist_bytes_match_restated_saveparams():
    arrays = _arrays()
    assert _write_blob(arrays) == ndarray_list.save_params(arrays)


def test_ndlist_readers_agree():
    arrays = _arrays()
    blob = ndarray_list.save_params(arrays)
    a = tf.parse_ndarray_list(blob, copy=True)
    b = ndarray_list.load_params(blob)
    for n, v in arrays:
        np.testing.assert_array_equal(a[n], v)
        np.testing.assert_array_equal(b[n], v)
        assert a[n].dtype == v.dtype and a[n].shape == v.shape


def test_c_parser():
    lib = _lib.load()
    arrays = _arrays()
    blob = np.frombuffer(ndarray_list.save_params(arrays), dtype=np.uint8).copy()
    metas = (_lib.tk_array_meta * 8)()
    offs = (ctypes.c_int64 * 8)()
    shapes = (ctypes.c_int64 * 64)()
    n = ctypes.c_int()
    _lib.check(lib.tk_ndlist_parse(ctypes.c_void_p(blob.ctypes.data), blob.size, 8, metas, offs, shapes, 64,
                                   ctypes.byref(n)))
    assert n.value == len(arrays)
    for i, (name, a) in enumerate(arrays):
        assert metas[i].ndim == a.ndim
        assert tuple(metas[i].shape[k] for k in range(a.ndim)) == a.shape
        got = blob[offs[i]:offs[i] + a.nbytes].view(a.dtype).reshape(a.shape)
        np.testing.assert_array_equal(got, a)


def test_trace_container_roundtrip(tmp_path):
    params = [("w", np.arange(24, dtype=np.int8).reshape(2, 3, 4))]
    records = [("data", np.arange(10, dtype=np.int8)), ("%0", np.arange(6, dtype=np.int32).reshape(2, 3) - 3)]
    meta = {"format": "tachikoma-trace", "model": "t", "sample_offset": 128, "ops": []}
    lay = tf.TraceLayout.compute(tf.header_json(meta), [(n, a.shape, str(a.dtype)) for n, a in params],
                                 [(n, a.shape, str(a.dtype)) for n, a in records])
    img = np.zeros(lay.total, dtype=np.uint8)
    lay.write_headers(img.ctypes.data, lay.total)
    for (n, a), off in zip(params, lay.param_offsets):
        img[off:off + a.nbytes] = np.frombuffer(a.tobytes(), np.uint8)
    for (n, a), off in zip(records, lay.record_offsets):
        img[off:off + a.nbytes] = np.frombuffer(a.tobytes(), np.uint8)
    assert lay.param_offsets[0] >= 4096 and min(lay.record_offsets) % 1 == 0
    path = str(tmp_path / "t.tkt")
    tf.write_file(path, img.ctypes.data, lay.total)
    tr = tf.read_trace(path, copy=True)
    assert tr.meta["sample_offset"] == 128
    for n, a in params:
        np.testing.assert_array_equal(tr.params[n], a)
    for n, a in records:
        np.testing.assert_array_equal(tr.records[n], a)
    # the params / records sections are plain NDArray-list blobs (LoadParams-compatible)
    raw = open(path, "rb").read()
    import struct
    _, _, _, po, ps, ro, rs = struct.unpack_from("<7Q", raw, 0)
    np.testing.assert_array_equal(ndarray_list.load_params(raw[ro:ro + rs])["%0"], records[1][1])

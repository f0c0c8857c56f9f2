"""The OpenMP C restatement (oracle/qnn_ref.c) equals the numpy oracle bit for bit."""
import numpy as np
import pytest

import oracle
from oracle import graph_ref
from oracle import qnn_ref as ref


@pytest.fixture(scope="module", autouse=True)
def _built():
    oracle.build_c()


def _rand(rng, shape, dtype):
    info = np.iinfo(dtype)
    return rng.integers(info.min, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


@pytest.mark.parametrize("case", [
    (2, 8, 9, 9, 16, 3, 1, (1, 1, 1, 1), 1, 1, "int8", "int8", -3, 0),
    (1, 3, 17, 15, 8, 7, 2, (3, 3, 3, 3), 1, 1, "int8", "int8", 5, 0),
    (1, 6, 10, 11, 6, 3, 2, (0, 1, 1, 0), 2, 6, "uint8", "int8", 130, 2),
    (2, 8, 8, 8, 12, 3, 1, (1, 1, 1, 1), 1, 4, "uint8", "uint8", 128, 127),
])
def test_conv_c_matches_numpy(case):
    n, c, h, w, o, k, s, pad, d, g, dx, dw_, za, zw = case
    rng = np.random.default_rng(1)
    x = _rand(rng, (n, c, h, w), dx)
    wt = _rand(rng, (o, c // g, k, k), dw_)
    attrs = {"strides": (s, s), "padding": pad, "dilation": (d, d), "groups": g}
    got = graph_ref._conv_c(x, wt, za, zw, attrs, 4)
    exp = ref.qnn_conv2d(x, wt, za, zw, strides=(s, s), padding=pad, dilation=(d, d), groups=g)
    np.testing.assert_array_equal(got, exp)


def test_dense_c_matches_numpy():
    rng = np.random.default_rng(2)
    for dx, dw_, za, zw in (("int8", "int8", -3, 0), ("uint8", "int8", 100, -1), ("int8", "uint8", 0, 128)):
        x = _rand(rng, (7, 33), dx)
        w = _rand(rng, (5, 33), dw_)
        np.testing.assert_array_equal(graph_ref._dense_c(x, w, za, zw, 2), ref.qnn_dense(x, w, za, zw))
    x = _rand(rng, (3, 10), "int8")
    w = _rand(rng, (4, 10), "int8")
    zv = np.array([1, -2, 3, 0], np.int32)
    np.testing.assert_array_equal(graph_ref._dense_c(x, w, 2, zv, 2), ref.qnn_dense(x, w, 2, zv))


def test_graph_numpy_vs_c_lenet():
    from tachikoma_amd import zoo
    m = zoo.lenet5(batch=2)
    x = m.random_input()
    a = graph_ref.calibrate(m.mod, m.params, {"data": x}, backend="numpy")
    b = graph_ref.calibrate(m.mod, m.params, {"data": x}, backend="c", threads=2)
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])

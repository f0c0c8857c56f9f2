"""Relay operators on the integer trace path (names and argument order as in tvm.relay).

Each constructor type-checks eagerly (the analogue of Relay's type relations,
e.g. ``src/relay/qnn/op/requantize.cc:465-514``) and returns a ``Call``.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np

from .expr import Call, Constant, Expr, TensorType, const

INT_DTYPES = ("int8", "uint8", "int16", "uint16", "int32", "uint32", "int64", "uint64")


def _tuple2(v) -> Tuple[int, int]:
    if isinstance(v, (int, np.integer)):
        return (int(v), int(v))
    v = tuple(int(x) for x in v)
    return v if len(v) == 2 else (v[0], v[0])


def get_pad_tuple2d(padding) -> Tuple[int, int, int, int]:
    """Relay padding normalisation (python/tvm/relay/op/nn/utils.py get_pad_tuple2d):
    int → all four; (h, w) → (h, w, h, w); (t, l, b, r) as is."""
    if isinstance(padding, (int, np.integer)):
        p = int(padding)
        return (p, p, p, p)
    p = tuple(int(x) for x in padding)
    if len(p) == 1:
        return (p[0],) * 4
    if len(p) == 2:
        return (p[0], p[1], p[0], p[1])
    if len(p) == 4:
        return p
    raise ValueError(f"bad padding {padding}")


def _check_int(e: Expr, what: str):
    if e.dtype not in INT_DTYPES:
        raise TypeError(f"{what}: integer tensor expected, got {e.dtype}")


# ---------------------------------------------------------------- nn.* / elementwise

def bias_add(data: Expr, bias: Expr, axis: int = 1) -> Call:
    ax = axis if axis >= 0 else len(data.shape) + axis
    if bias.shape != (data.shape[ax],):
        raise TypeError(f"nn.bias_add: bias {bias.shape} does not match axis {axis} of {data.shape}")
    if bias.dtype != data.dtype:
        raise TypeError("nn.bias_add: dtype mismatch")
    return Call("nn.bias_add", [data, bias], {"axis": axis}, data.checked_type)


def add(lhs: Expr, rhs: Expr) -> Call:
    """``relay.add`` (python/tvm/relay/op/tensor.py; topi broadcast_add): on the integer trace
    path the broadcast operand is a per-channel vector along axis 1 (a bias given as [C, 1, 1]
    or [C], the way frontends and the reference's tachikoma tests write it)."""
    if lhs.dtype != rhs.dtype:
        raise TypeError("add: dtype mismatch")
    nd, rs = len(lhs.shape), tuple(rhs.shape)
    padded = (1,) * (nd - len(rs)) + rs if len(rs) <= nd else None
    if nd < 2 or padded is None or padded[1] != lhs.shape[1] or any(d != 1 for i, d in enumerate(padded) if i != 1):
        raise NotImplementedError(f"add: only a per-channel vector broadcast along axis 1 ({lhs.shape} + {rs})")
    return Call("add", [lhs, rhs], {}, lhs.checked_type)


def clip(a: Expr, a_min: float, a_max: float) -> Call:
    return Call("clip", [a], {"a_min": float(a_min), "a_max": float(a_max)}, a.checked_type)


def relu(data: Expr) -> Call:
    return Call("nn.relu", [data], {}, data.checked_type)


def cast(data: Expr, dtype: str) -> Call:
    return Call("cast", [data], {"dtype": str(np.dtype(dtype))}, TensorType(data.shape, str(np.dtype(dtype))))


def max_pool2d(data: Expr, pool_size=(1, 1), strides=(1, 1), dilation=(1, 1), padding=(0, 0), layout="NCHW",
               out_layout="", ceil_mode=False) -> Call:
    return _pool("nn.max_pool2d", data, pool_size, strides, dilation, padding, layout, ceil_mode, {})


def avg_pool2d(data: Expr, pool_size=(1, 1), strides=(1, 1), dilation=(1, 1), padding=(0, 0), layout="NCHW",
               out_layout="", ceil_mode=False, count_include_pad=False) -> Call:
    return _pool("nn.avg_pool2d", data, pool_size, strides, dilation, padding, layout, ceil_mode,
                 {"count_include_pad": bool(count_include_pad)})


def _pool(name, data, pool_size, strides, dilation, padding, layout, ceil_mode, extra) -> Call:
    if layout != "NCHW":
        raise NotImplementedError(f"{name}: only NCHW layout is supported")
    if ceil_mode:
        raise NotImplementedError(f"{name}: ceil_mode is not supported")
    _check_int(data, name)
    kh, kw = _tuple2(pool_size)
    sh, sw = _tuple2(strides)
    dh, dw = _tuple2(dilation)
    pt, pl, pb, pr = get_pad_tuple2d(padding)
    n, c, h, w = data.shape
    oh = (h + pt + pb - dh * (kh - 1) - 1) // sh + 1
    ow = (w + pl + pr - dw * (kw - 1) - 1) // sw + 1
    attrs = {"pool_size": (kh, kw), "strides": (sh, sw), "dilation": (dh, dw), "padding": (pt, pl, pb, pr),
             "layout": layout, "ceil_mode": False}
    attrs.update(extra)
    return Call(name, [data], attrs, TensorType((n, c, oh, ow), data.dtype))


def global_avg_pool2d(data: Expr, layout="NCHW", out_layout="") -> Call:
    if layout != "NCHW":
        raise NotImplementedError("nn.global_avg_pool2d: only NCHW layout is supported")
    _check_int(data, "nn.global_avg_pool2d")
    n, c, _, _ = data.shape
    return Call("nn.global_avg_pool2d", [data], {"layout": layout}, TensorType((n, c, 1, 1), data.dtype))


def batch_flatten(data: Expr) -> Call:
    n = data.shape[0]
    rest = int(np.prod(data.shape[1:])) if len(data.shape) > 1 else 1
    return Call("nn.batch_flatten", [data], {}, TensorType((n, rest), data.dtype))


def reshape(data: Expr, newshape) -> Call:
    total = int(np.prod(data.shape))
    shape = list(int(s) for s in newshape)
    if -1 in shape:
        k = shape.index(-1)
        rest = int(np.prod([s for i, s in enumerate(shape) if i != k]))
        shape[k] = total // rest
    if int(np.prod(shape)) != total:
        raise TypeError(f"reshape: {data.shape} -> {newshape}")
    return Call("reshape", [data], {"newshape": tuple(shape)}, TensorType(tuple(shape), data.dtype))

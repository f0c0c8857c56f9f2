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


def _broadcast_shape(name: str, a, b) -> Tuple[int, ...]:
    try:
        shape = np.broadcast_shapes(tuple(a), tuple(b))
    except ValueError as e:
        raise TypeError(f"{name}: {tuple(a)} and {tuple(b)} do not broadcast") from e
    return tuple(int(d) for d in shape)


def _broadcast(name: str, lhs: Expr, rhs: Expr) -> TensorType:
    """Relay's BroadcastRel (src/relay/op/type_relations.cc): numpy broadcasting, equal dtypes."""
    if lhs.dtype != rhs.dtype:
        raise TypeError(f"{name}: dtype mismatch {lhs.dtype} vs {rhs.dtype}")
    return TensorType(_broadcast_shape(name, lhs.shape, rhs.shape), lhs.dtype)


def add(lhs: Expr, rhs: Expr) -> Call:
    """``relay.add`` (python/tvm/relay/op/tensor.py; topi broadcast_add), numpy broadcasting.
    The device runs same-shape, scalar and per-channel-vector (a bias given as [C, 1, 1] or
    [C], the way frontends and the reference's tachikoma tests write it) operands."""
    return Call("add", [lhs, rhs], {}, _broadcast("add", lhs, rhs))


def multiply(lhs: Expr, rhs: Expr) -> Call:
    """``relay.multiply`` (topi broadcast_mul)."""
    return Call("multiply", [lhs, rhs], {}, _broadcast("multiply", lhs, rhs))


def right_shift(lhs: Expr, rhs: Expr) -> Call:
    """``relay.right_shift`` (arithmetic shift for signed types)."""
    _check_int(lhs, "right_shift")
    return Call("right_shift", [lhs, rhs], {}, _broadcast("right_shift", lhs, rhs))


def left_shift(lhs: Expr, rhs: Expr) -> Call:
    """``relay.left_shift`` (wraps in the operand type)."""
    _check_int(lhs, "left_shift")
    return Call("left_shift", [lhs, rhs], {}, _broadcast("left_shift", lhs, rhs))


def round(data: Expr) -> Call:  # noqa: A001  (relay.round)
    """``relay.round``: llvm.round, halves away from zero."""
    if data.dtype in INT_DTYPES:
        raise TypeError("round: float tensor expected")
    return Call("round", [data], {}, data.checked_type)


def fixed_point_multiply(data: Expr, multiplier: int, shift: int) -> Call:
    """``relay.fixed_point_multiply`` (topi/math.py:644-673 → tir.q_multiply_shift(x, m, 31, s))."""
    _check_int(data, "fixed_point_multiply")
    return Call("fixed_point_multiply", [data], {"multiplier": int(multiplier), "shift": int(shift)},
                data.checked_type)


def stop_fusion(data: Expr) -> Call:
    """``annotation.stop_fusion``: identity that ends a fusion group."""
    return Call("annotation.stop_fusion", [data], {}, data.checked_type)


def cast_hint(data: Expr, dtype: str) -> Call:
    """``annotation.cast_hint``: identity carrying the dtype the quantizer will cast to."""
    return Call("annotation.cast_hint", [data], {"dtype": str(np.dtype(dtype))}, data.checked_type)


def conv2d(data: Expr, weight: Expr, strides=(1, 1), padding=(0, 0), dilation=(1, 1), groups=1, channels=None,
           kernel_size=None, data_layout="NCHW", kernel_layout="OIHW", out_layout="", out_dtype="") -> Call:
    """``relay.nn.conv2d`` (NCHW/OIHW): float32, or int8 x int8 -> out_dtype (the realized
    quantized graph, realize.cc:147-174)."""
    if data_layout != "NCHW" or kernel_layout != "OIHW":
        raise NotImplementedError("nn.conv2d: only NCHW/OIHW layouts are supported")
    n, c, h, w = data.shape
    o, cg, kh, kw = weight.shape
    sh, sw = _tuple2(strides)
    dh, dw = _tuple2(dilation)
    pt, pl, pb, pr = get_pad_tuple2d(padding)
    if c != cg * int(groups) or o % int(groups):
        raise TypeError(f"nn.conv2d: channels {c} / groups {groups} vs weight {weight.shape}")
    oh = (h + pt + pb - dh * (kh - 1) - 1) // sh + 1
    ow = (w + pl + pr - dw * (kw - 1) - 1) // sw + 1
    odt = str(np.dtype(out_dtype)) if out_dtype else data.dtype
    attrs = {"strides": (sh, sw), "padding": (pt, pl, pb, pr), "dilation": (dh, dw), "groups": int(groups),
             "channels": o, "kernel_size": (kh, kw), "data_layout": "NCHW", "kernel_layout": "OIHW",
             "out_dtype": odt}
    return Call("nn.conv2d", [data, weight], attrs, TensorType((n, o, oh, ow), odt))


def dense(data: Expr, weight: Expr, units=None, out_dtype="") -> Call:
    """``relay.nn.dense``: data [M, K] x weight [N, K]^T."""
    m, k = data.shape
    nn_, k2 = weight.shape
    if k != k2:
        raise TypeError(f"nn.dense: {data.shape} x {weight.shape}")
    odt = str(np.dtype(out_dtype)) if out_dtype else data.dtype
    return Call("nn.dense", [data, weight], {"units": nn_, "out_dtype": odt}, TensorType((m, nn_), odt))


def transpose(data: Expr, axes=None) -> Call:
    """``relay.transpose`` (src/relay/op/tensor/transform.cc TransposeRel): axes=None reverses."""
    nd = len(data.shape)
    ax = tuple(range(nd))[::-1] if axes is None else tuple(int(a) + nd if int(a) < 0 else int(a) for a in axes)
    if sorted(ax) != list(range(nd)):
        raise TypeError(f"transpose: {axes} is not a permutation of {nd} axes")
    return Call("transpose", [data], {"axes": ax}, TensorType(tuple(data.shape[a] for a in ax), data.dtype))


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
    n, c, _, _ = data.shape
    return Call("nn.global_avg_pool2d", [data], {"layout": layout}, TensorType((n, c, 1, 1), data.dtype))


def batch_flatten(data: Expr) -> Call:
    n = data.shape[0]
    rest = int(np.prod(data.shape[1:])) if len(data.shape) > 1 else 1
    return Call("nn.batch_flatten", [data], {}, TensorType((n, rest), data.dtype))


def reshape(data: Expr, newshape) -> Call:
    """``relay.reshape`` with Relay's special values 0 (copy the input dimension) and -1 (infer)
    (src/relay/op/tensor/transform.cc InferNewShape)."""
    total = int(np.prod(data.shape))
    shape = [int(data.shape[i]) if int(s) == 0 else int(s) for i, s in enumerate(newshape)]
    if -1 in shape:
        k = shape.index(-1)
        rest = int(np.prod([s for i, s in enumerate(shape) if i != k]))
        shape[k] = total // rest
    if int(np.prod(shape)) != total:
        raise TypeError(f"reshape: {data.shape} -> {newshape}")
    return Call("reshape", [data], {"newshape": tuple(shape)}, TensorType(tuple(shape), data.dtype))


def pad(data: Expr, pad_width, pad_value=0.0, pad_mode: str = "constant") -> Call:
    """``relay.nn.pad`` (src/relay/op/nn/pad.cc, topi/nn/pad.py), constant mode: ``pad_width`` is
    one (before, after) pair per axis; the pad value (a scalar, or a scalar constant expression as
    the text form writes it: ``nn.pad(%x, 0f, pad_width=...)``) is cast to the data's dtype."""
    if pad_mode != "constant":
        raise NotImplementedError("nn.pad: only pad_mode='constant' is supported")
    pw = tuple((int(b), int(a)) for b, a in pad_width)
    if len(pw) != len(data.shape) or any(b < 0 or a < 0 for b, a in pw):
        raise TypeError(f"nn.pad: pad_width {pad_width} for a {len(data.shape)}-D tensor")
    if isinstance(pad_value, Constant):
        if pad_value.data.ndim != 0:
            raise TypeError("nn.pad: the pad value must be a scalar")
        v = pad_value.data.item()
    elif isinstance(pad_value, Expr):
        raise TypeError("nn.pad: the pad value must be a constant")
    else:
        v = pad_value
    pv = const(np.asarray(v).astype(data.dtype), data.dtype)
    shape = tuple(int(d) + b + a for d, (b, a) in zip(data.shape, pw))
    return Call("nn.pad", [data, pv], {"pad_width": pw, "pad_mode": "constant"}, TensorType(shape, data.dtype))


class TupleGetItem(Expr):
    """A field of a multi-output op (``%0.0``).  Only ``nn.batch_norm``'s normalised output (field
    0) exists on this path: the op's node IS that output, so field 0 resolves to it."""


class BatchNormOutputs:
    """What ``relay.nn.batch_norm`` returns (the reference's TupleWrapper of (out, moving_mean,
    moving_var)); inference graphs use field 0 only."""

    def __init__(self, call: Call):
        self.call = call

    def __getitem__(self, i: int) -> Call:
        if i != 0:
            raise NotImplementedError("nn.batch_norm: only the normalised output (field 0) is supported")
        return self.call

    def astuple(self) -> Call:
        return self.call


def batch_norm(data: Expr, gamma: Expr, beta: Expr, moving_mean: Expr, moving_var: Expr, axis: int = 1,
               epsilon: float = 1e-5, center: bool = True, scale: bool = True) -> BatchNormOutputs:
    """``relay.nn.batch_norm`` (src/relay/op/nn/nn.cc BatchNormRel): float data, four per-channel
    vectors along ``axis``.  Graphs holding it are rewritten by ``transform.simplify_inference``
    (``relay.build`` and ``relay.quantize`` run it first, as the reference's pass prefix and
    prerequisite_optimize do)."""
    ax = axis if axis >= 0 else len(data.shape) + axis
    c = data.shape[ax]
    for name, v in (("gamma", gamma), ("beta", beta), ("moving_mean", moving_mean), ("moving_var", moving_var)):
        if tuple(v.shape) != (c,) or v.dtype != data.dtype:
            raise TypeError(f"nn.batch_norm: {name} {v.shape} {v.dtype} vs {c} channels of {data.dtype}")
    attrs = {"axis": int(axis), "epsilon": float(epsilon), "center": bool(center), "scale": bool(scale)}
    return BatchNormOutputs(Call("nn.batch_norm", [data, gamma, beta, moving_mean, moving_var], attrs,
                                 data.checked_type))

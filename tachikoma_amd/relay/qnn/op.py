"""``relay.qnn.op`` constructors (python/tvm/relay/qnn/op/qnn.py signatures).

Scales and zero points are Relay constants (python numbers are wrapped with
``relay.const`` the way the reference's tests do); a rank-0 scale is
per-tensor, a 1-D scale per-axis (``IsConstScalar``, pattern_utils.h:272-278).
"""
from __future__ import annotations

import contextlib
import threading
from typing import Optional

import numpy as np

from ..expr import Call, Constant, Expr, TensorType, const
from ..op import _check_int, _tuple2, get_pad_tuple2d

_cfg = threading.local()


def _cfg_stack():
    if not hasattr(_cfg, "stack"):
        _cfg.stack = []
    return _cfg.stack


@contextlib.contextmanager
def requantize_config(rounding: Optional[str] = None, compute_dtype: Optional[str] = None):
    """``relay.qnn.op.requantize_config`` scope (src/relay/qnn/op/requantize_config.cc:35-89).

    Values apply to requantize ops whose own argument is "None"; per-op arguments win
    (SelectRequntizeParameter, src/relay/qnn/utils.cc:218-229).
    """
    _cfg_stack().append({"rounding": rounding, "compute_dtype": compute_dtype})
    try:
        yield
    finally:
        _cfg_stack().pop()


def current_requantize_config():
    st = _cfg_stack()
    return st[-1] if st else {"rounding": None, "compute_dtype": None}


def _c(v, dtype):
    if isinstance(v, Expr):
        return v
    return const(v, dtype)


def requantize(data: Expr, input_scale, input_zero_point, output_scale, output_zero_point, axis: int = -1,
               rounding: str = "None", compute_dtype: str = "None", out_dtype: str = "int8") -> Call:
    _check_int(data, "qnn.requantize")
    input_scale = _c(input_scale, "float32")
    output_scale = _c(output_scale, "float32")
    input_zero_point = _c(input_zero_point, "int32")
    output_zero_point = _c(output_zero_point, "int32")
    if output_scale.checked_type.shape != ():
        raise TypeError("qnn.requantize: output_scale must be a scalar")
    ax = axis if axis >= 0 else len(data.shape) + axis
    if input_scale.checked_type.shape not in ((),) and len(data.shape) > 0:
        if input_scale.checked_type.shape[0] != data.shape[ax]:
            raise TypeError("qnn.requantize: per-axis scale length does not match the axis")
    cfg = current_requantize_config()
    attrs = {"axis": axis, "rounding": rounding, "compute_dtype": compute_dtype, "out_dtype": str(np.dtype(out_dtype)),
             "cfg_rounding": cfg["rounding"], "cfg_compute_dtype": cfg["compute_dtype"]}
    return Call("qnn.requantize", [data, input_scale, input_zero_point, output_scale, output_zero_point], attrs,
                TensorType(data.shape, str(np.dtype(out_dtype))))


def conv2d(data: Expr, kernel: Expr, input_zero_point, kernel_zero_point, input_scale, kernel_scale, kernel_size,
           channels, strides=(1, 1), padding=(0, 0), dilation=(1, 1), groups: int = 1, data_layout="NCHW",
           kernel_layout="OIHW", out_layout="", out_dtype="int32") -> Call:
    if data_layout != "NCHW" or kernel_layout != "OIHW":
        raise NotImplementedError("qnn.conv2d: NCHW/OIHW only (the layout the reference traces)")
    if str(np.dtype(out_dtype)) != "int32":
        raise NotImplementedError("qnn.conv2d: out_dtype must be int32")
    _check_int(data, "qnn.conv2d")
    _check_int(kernel, "qnn.conv2d")
    n, c, h, w = data.shape
    o, cg, kh, kw = kernel.shape
    if c != cg * groups:
        raise TypeError(f"qnn.conv2d: {c} input channels vs kernel {kernel.shape} with groups={groups}")
    sh, sw = _tuple2(strides)
    dh, dw = _tuple2(dilation)
    pt, pl, pb, pr = get_pad_tuple2d(padding)
    if tuple(_tuple2(kernel_size)) != (kh, kw):
        raise TypeError("qnn.conv2d: kernel_size does not match the kernel shape")
    oh = (h + pt + pb - dh * (kh - 1) - 1) // sh + 1
    ow = (w + pl + pr - dw * (kw - 1) - 1) // sw + 1
    attrs = {"strides": (sh, sw), "padding": (pt, pl, pb, pr), "dilation": (dh, dw), "groups": int(groups),
             "channels": int(channels) if channels is not None else o, "kernel_size": (kh, kw),
             "data_layout": data_layout, "kernel_layout": kernel_layout, "out_dtype": "int32"}
    args = [data, kernel, _c(input_zero_point, "int32"), _c(kernel_zero_point, "int32"),
            _c(input_scale, "float32"), _c(kernel_scale, "float32")]
    return Call("qnn.conv2d", args, attrs, TensorType((n, o, oh, ow), "int32"))


def dense(data: Expr, weight: Expr, input_zero_point, kernel_zero_point, input_scale, kernel_scale, units,
          out_dtype="int32") -> Call:
    if str(np.dtype(out_dtype)) != "int32":
        raise NotImplementedError("qnn.dense: out_dtype must be int32")
    _check_int(data, "qnn.dense")
    _check_int(weight, "qnn.dense")
    m, k = data.shape
    nn_, k2 = weight.shape
    if k != k2 or (units is not None and int(units) != nn_):
        raise TypeError(f"qnn.dense: {data.shape} x {weight.shape} (units={units})")
    args = [data, weight, _c(input_zero_point, "int32"), _c(kernel_zero_point, "int32"),
            _c(input_scale, "float32"), _c(kernel_scale, "float32")]
    return Call("qnn.dense", args, {"units": nn_, "out_dtype": "int32"}, TensorType((m, nn_), "int32"))


def add(lhs: Expr, rhs: Expr, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
        output_zero_point, lhs_axis: int = -1, rhs_axis: int = -1) -> Call:
    _check_int(lhs, "qnn.add")
    if lhs.shape != rhs.shape or lhs.dtype != rhs.dtype:
        raise NotImplementedError("qnn.add: same-shape, same-dtype operands only")
    args = [lhs, rhs, _c(lhs_scale, "float32"), _c(lhs_zero_point, "int32"), _c(rhs_scale, "float32"),
            _c(rhs_zero_point, "int32"), _c(output_scale, "float32"), _c(output_zero_point, "int32")]
    return Call("qnn.add", args, {"lhs_axis": lhs_axis, "rhs_axis": rhs_axis}, lhs.checked_type)

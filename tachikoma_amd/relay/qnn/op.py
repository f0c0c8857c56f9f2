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

from ..expr import Call, Constant, Expr, TensorType, Tuple, const
from ..op import _broadcast_shape, _check_int, _tuple2, get_pad_tuple2d
from ..op import reshape as _reshape

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


KERNEL_LAYOUTS = ("OIHW", "HWIO", "OHWI", "HWOI")


def conv2d(data: Expr, kernel: Expr, input_zero_point, kernel_zero_point, input_scale, kernel_scale, kernel_size,
           channels, strides=(1, 1), padding=(0, 0), dilation=(1, 1), groups: int = 1, data_layout="NCHW",
           kernel_layout="OIHW", out_layout="", out_dtype="int32") -> Call:
    """``qnn.conv2d`` with the layouts the reference's QNN conv accepts
    (src/relay/qnn/op/convolution.cc:718-722): NCHW / NHWC data, OIHW / HWIO / OHWI / HWOI kernel;
    the output is in the data layout (Conv2DRel's default out_layout)."""
    if data_layout not in ("NCHW", "NHWC") or kernel_layout not in KERNEL_LAYOUTS:
        raise NotImplementedError(f"qnn.conv2d: data layout {data_layout} / kernel layout {kernel_layout}: "
                                  f"NCHW or NHWC data with {', '.join(KERNEL_LAYOUTS)} kernels")
    if out_layout not in ("", data_layout):
        raise NotImplementedError("qnn.conv2d: out_layout must be the data layout")
    if str(np.dtype(out_dtype)) != "int32":
        raise NotImplementedError("qnn.conv2d: out_dtype must be int32")
    _check_int(data, "qnn.conv2d")
    _check_int(kernel, "qnn.conv2d")
    if data_layout == "NCHW":
        n, c, h, w = data.shape
    else:
        n, h, w, c = data.shape
    ks = dict(zip(kernel_layout, kernel.shape))
    o, cg, kh, kw = ks["O"], ks["I"], ks["H"], ks["W"]
    multiplier = 1
    if groups > 1 and groups == c and o == groups and cg > 1:
        # Conv2DRel's depthwise form (src/relay/op/nn/convolution.cc:243-274): the OIHW-space weight is
        # (C, multiplier, KH, KW) and output channel c * multiplier + m reads weight[c, m]
        multiplier = cg
        if channels is not None and int(channels) != c * multiplier:
            raise TypeError(f"qnn.conv2d: depthwise kernel {kernel.shape} gives {c * multiplier} channels, "
                            f"not {channels}")
        o, cg = c * multiplier, 1
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
    if multiplier > 1:
        attrs["depthwise_multiplier"] = multiplier
    args = [data, kernel, _c(input_zero_point, "int32"), _c(kernel_zero_point, "int32"),
            _c(input_scale, "float32"), _c(kernel_scale, "float32")]
    shape = (n, o, oh, ow) if data_layout == "NCHW" else (n, oh, ow, o)
    return Call("qnn.conv2d", args, attrs, TensorType(shape, "int32"))


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


def _binary(name: str, lhs: Expr, rhs: Expr, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
            output_zero_point, lhs_axis: int, rhs_axis: int) -> Call:
    """QNN_REGISTER_BINARY_OP operands (src/relay/qnn/op/op_common.h:231-320, QnnBroadcastRel):
    numpy broadcasting of equal-dtype operands; scales / zero points rank-0 (per-tensor) or one
    per index of ``lhs_axis`` / ``rhs_axis`` of that operand."""
    _check_int(lhs, name)
    if lhs.dtype != rhs.dtype:
        raise TypeError(f"{name}: dtype mismatch {lhs.dtype} vs {rhs.dtype}")
    if lhs.dtype not in ("int8", "uint8", "int16", "int32"):
        raise TypeError(f"{name}: int8, uint8, int16 or int32 operands expected, got {lhs.dtype}")
    shape = _broadcast_shape(name, lhs.shape, rhs.shape)
    args = [lhs, rhs, _c(lhs_scale, "float32"), _c(lhs_zero_point, "int32"), _c(rhs_scale, "float32"),
            _c(rhs_zero_point, "int32"), _c(output_scale, "float32"), _c(output_zero_point, "int32")]
    for side, x, ax, (si, zi) in (("lhs", lhs, lhs_axis, (2, 3)), ("rhs", rhs, rhs_axis, (4, 5))):
        nd = len(x.shape)
        a = 0 if nd <= 1 else (nd + ax if ax < 0 else ax)
        for k in (si, zi):
            p = args[k].checked_type.shape
            if p != () and (nd and not (0 <= a < nd) or p != ((x.shape[a] if nd else 1),)):
                raise TypeError(f"{name}: {side} parameter of shape {p} does not match axis {ax} of {x.shape}")
    if args[6].checked_type.shape != () or args[7].checked_type.shape != ():
        raise TypeError(f"{name}: output scale / zero point must be scalars")
    cfg = current_requantize_config()
    attrs = {"lhs_axis": int(lhs_axis), "rhs_axis": int(rhs_axis), "cfg_rounding": cfg["rounding"],
             "cfg_compute_dtype": cfg["compute_dtype"]}
    return Call(name, args, attrs, TensorType(shape, lhs.dtype))


def add(lhs: Expr, rhs: Expr, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
        output_zero_point, lhs_axis: int = -1, rhs_axis: int = -1) -> Call:
    """``qnn.add`` (src/relay/qnn/op/add.cc:40-96)."""
    return _binary("qnn.add", lhs, rhs, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
                   output_zero_point, lhs_axis, rhs_axis)


def subtract(lhs: Expr, rhs: Expr, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
             output_zero_point, lhs_axis: int = -1, rhs_axis: int = -1) -> Call:
    """``qnn.subtract`` (src/relay/qnn/op/subtract.cc:40-94)."""
    return _binary("qnn.subtract", lhs, rhs, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
                   output_zero_point, lhs_axis, rhs_axis)


def mul(lhs: Expr, rhs: Expr, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
        output_zero_point, lhs_axis: int = -1, rhs_axis: int = -1) -> Call:
    """``qnn.mul`` (src/relay/qnn/op/mul.cc:43-159)."""
    return _binary("qnn.mul", lhs, rhs, lhs_scale, lhs_zero_point, rhs_scale, rhs_zero_point, output_scale,
                   output_zero_point, lhs_axis, rhs_axis)


def _as_tuple(v, dtype) -> Tuple:
    if isinstance(v, Tuple):
        return v
    return Tuple([_c(x, dtype) for x in v])


def concatenate(data, input_scales, input_zero_points, output_scale, output_zero_point, axis: int) -> Call:
    """``qnn.concatenate`` (src/relay/qnn/op/concatenate.cc:39-97 QnnConcatenateRel, :137-144): a
    tuple of equal-rank, equal-dtype tensors that agree outside ``axis``; one scalar scale and zero
    point per input, scalar output params."""
    data = data if isinstance(data, Tuple) else Tuple(list(data))
    scales, zps = _as_tuple(input_scales, "float32"), _as_tuple(input_zero_points, "int32")
    if not data.fields or len(scales) != len(data) or len(zps) != len(data):
        raise TypeError("qnn.concatenate: one scale and one zero point per input tensor")
    for f in scales.fields + zps.fields:
        if f.checked_type.shape != ():
            raise TypeError("qnn.concatenate: input scales / zero points must be scalars")
    first = data.fields[0]
    nd = len(first.shape)
    ax = axis + nd if axis < 0 else axis
    if not 0 <= ax < nd:
        raise TypeError(f"qnn.concatenate: axis {axis} out of range for rank {nd}")
    total = 0
    for x in data.fields:
        _check_int(x, "qnn.concatenate")
        if len(x.shape) != nd or x.dtype != first.dtype or any(
                x.shape[d] != first.shape[d] for d in range(nd) if d != ax):
            raise TypeError(f"qnn.concatenate: {x.shape} {x.dtype} does not concatenate with "
                            f"{first.shape} {first.dtype} on axis {axis}")
        total += x.shape[ax]
    shape = tuple(total if d == ax else first.shape[d] for d in range(nd))
    out_s, out_z = _c(output_scale, "float32"), _c(output_zero_point, "int32")
    if out_s.checked_type.shape != () or out_z.checked_type.shape != ():
        raise TypeError("qnn.concatenate: output scale / zero point must be scalars")
    cfg = current_requantize_config()
    attrs = {"axis": int(axis), "cfg_rounding": cfg["rounding"], "cfg_compute_dtype": cfg["compute_dtype"]}
    return Call("qnn.concatenate", [data, scales, zps, out_s, out_z], attrs, TensorType(shape, first.dtype))


def _axis_param(p: Expr, x_shape, axis: int, what: str):
    nd = len(x_shape)
    a = axis + nd if axis < 0 else axis
    shp = p.checked_type.shape
    if shp == () or int(np.prod(shp)) == 1:
        return
    if not (0 <= a < max(nd, 1)) or shp != (x_shape[a],):
        raise TypeError(f"{what}: parameter of shape {shp} does not match axis {axis} of {x_shape}")


def quantize(data: Expr, output_scale, output_zero_point, axis: int = -1, out_dtype: str = "int8") -> Call:
    """``qnn.quantize`` (src/relay/qnn/op/quantize.cc:39-111): float32 → int8 / uint8 / int16 / int32."""
    if data.dtype != "float32":
        raise TypeError(f"qnn.quantize: float32 data expected, got {data.dtype}")
    odt = str(np.dtype(out_dtype))
    if odt not in ("int8", "uint8", "int16", "int32"):
        raise TypeError(f"qnn.quantize: out_dtype must be int8, uint8, int16 or int32, got {odt}")
    s, z = _c(output_scale, "float32"), _c(output_zero_point, "int32")
    _axis_param(s, data.shape, axis, "qnn.quantize")
    _axis_param(z, data.shape, axis, "qnn.quantize")
    return Call("qnn.quantize", [data, s, z], {"axis": int(axis), "out_dtype": odt}, TensorType(data.shape, odt))


def dequantize(data: Expr, input_scale, input_zero_point, axis: int = -1) -> Call:
    """``qnn.dequantize`` (src/relay/qnn/op/dequantize.cc:39-94): int8 / uint8 / int16 / int32 → float32."""
    if data.dtype not in ("int8", "uint8", "int16", "int32"):
        raise TypeError(f"qnn.dequantize: int8, uint8, int16 or int32 data expected, got {data.dtype}")
    s, z = _c(input_scale, "float32"), _c(input_zero_point, "int32")
    _axis_param(s, data.shape, axis, "qnn.dequantize")
    _axis_param(z, data.shape, axis, "qnn.dequantize")
    return Call("qnn.dequantize", [data, s, z], {"axis": int(axis)}, TensorType(data.shape, "float32"))


# SQNN_DTYPE_TO_CODE (python/tvm/topi/nn/qnn.py:22-33): the simulated ops take their dtype as an
# int32 tensor, so a graph may choose it at run time
SQNN_DTYPE_TO_CODE = {"disable": 0, "int8": 1, "uint8": 2, "int32": 3}


def _sqnn(data: Expr, dtype, scale, zero_point, op: str):
    if data.dtype != "float32":
        raise TypeError(f"{op}: float32 data expected, got {data.dtype}")
    if isinstance(dtype, str):
        if dtype not in SQNN_DTYPE_TO_CODE:
            raise ValueError(f"{op}: dtype must be one of {sorted(SQNN_DTYPE_TO_CODE)}, got {dtype!r}")
        code = const(SQNN_DTYPE_TO_CODE[dtype], "int32")
    else:
        code = _c(dtype, "int32")
        if code.dtype != "int32" or int(np.prod(code.checked_type.shape)) != 1:
            raise TypeError(f"{op}: the dtype code must be one int32 value")
    # the constructor wraps both parameters in reshape(-1) (relay/qnn/op/qnn.py:253-255, 320-322)
    s = _reshape(_c(scale, "float32"), [-1])
    z = _reshape(_c(zero_point, "int32"), [-1])
    if s.dtype != "float32" or z.dtype != "int32":
        raise TypeError(f"{op}: float32 scale and int32 zero point expected")
    return code, s, z


def simulated_quantize(data: Expr, output_scale, output_zero_point, axis: int = -1, out_dtype="int8") -> Call:
    """``qnn.simulated_quantize`` (src/relay/qnn/op/simulated_quantize.cc:36-78, constructor
    python/tvm/relay/qnn/op/qnn.py:221-256): float32 → float32 holding the quantized values;
    ``out_dtype`` is a dtype name or an int32 tensor of an SQNN code, the scale / zero point a
    scalar or one value per channel along ``axis`` (taken modulo their length)."""
    code, s, z = _sqnn(data, out_dtype, output_scale, output_zero_point, "qnn.simulated_quantize")
    return Call("qnn.simulated_quantize", [data, code, s, z], {"axis": int(axis)}, TensorType(data.shape, data.dtype))


def simulated_call(op: str, data: Expr, dtype_code: Expr, scale: Expr, zero_point: Expr, axis: int = -1) -> Call:
    """The simulated op as Relay text spells it -- (data, dtype code, scale, zero point), the
    parameters already 1-D (MakeSimulatedQuantize / MakeSimulatedDequantize) -- for the parser."""
    if data.dtype != "float32":
        raise TypeError(f"{op}: float32 data expected, got {data.dtype}")
    return Call(op, [data, dtype_code, scale, zero_point], {"axis": int(axis)}, TensorType(data.shape, data.dtype))


def simulated_dequantize(data: Expr, input_scale, input_zero_point, axis: int = -1, in_dtype="int8") -> Call:
    """``qnn.simulated_dequantize`` (src/relay/qnn/op/simulated_dequantize.cc:36-76, constructor
    python/tvm/relay/qnn/op/qnn.py:288-323): float32 → float32, ``(x - zp) * scale``."""
    code, s, z = _sqnn(data, in_dtype, input_scale, input_zero_point, "qnn.simulated_dequantize")
    return Call("qnn.simulated_dequantize", [data, code, s, z], {"axis": int(axis)},
                TensorType(data.shape, data.dtype))


def _scalar_param(p: Expr, what: str) -> None:
    shp = p.checked_type.shape
    if shp != () and int(np.prod(shp)) != 1:
        raise TypeError(f"{what}: scale / zero point must be a scalar (or one element), got shape {shp}")


def leaky_relu(x: Expr, alpha: float, input_scale, input_zero_point, output_scale, output_zero_point) -> Call:
    """``qnn.leaky_relu`` (src/relay/qnn/op/leaky_relu.cc:33-77): int8 / uint8 data, scalar params,
    the output in the input's dtype."""
    if x.dtype not in ("int8", "uint8"):
        raise TypeError(f"qnn.leaky_relu: int8 or uint8 data expected, got {x.dtype}")
    args = [x, _c(input_scale, "float32"), _c(input_zero_point, "int32"), _c(output_scale, "float32"),
            _c(output_zero_point, "int32")]
    for p in args[1:]:
        if p.checked_type.shape != ():
            raise TypeError("qnn.leaky_relu: scales and zero points must be scalars")
    cfg = current_requantize_config()
    attrs = {"alpha": float(alpha), "cfg_rounding": cfg["rounding"], "cfg_compute_dtype": cfg["compute_dtype"]}
    return Call("qnn.leaky_relu", args, attrs, TensorType(x.shape, x.dtype))


# the unary ops of src/relay/qnn/op/unary_elementwise_op.cc:31-56 (QNN_CREATE_UNARY_ELEMENTWISE_OP);
# each is legalized to a 256-entry table lookup (python/tvm/relay/qnn/op/legalizations.py:54-86)
UNARY_OPS = ("qnn.sqrt", "qnn.rsqrt", "qnn.exp", "qnn.erf", "qnn.sigmoid", "qnn.hardswish", "qnn.tanh", "qnn.log",
             "qnn.abs")


def _unary(name: str, x: Expr, scale, zero_point, output_scale, output_zero_point) -> Call:
    """QnnUnaryElementwiseRel: int8 / uint8 data, scalar params, same dtype out."""
    if x.dtype not in ("int8", "uint8"):
        raise TypeError(f"{name}: int8 or uint8 data expected, got {x.dtype}")
    args = [x, _c(scale, "float32"), _c(zero_point, "int32"), _c(output_scale, "float32"),
            _c(output_zero_point, "int32")]
    for p in args[1:]:
        if p.checked_type.shape != ():
            raise TypeError(f"{name}: scales and zero points must be scalars")
    return Call(name, args, {}, TensorType(x.shape, x.dtype))


def sqrt(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.sqrt", x, scale, zero_point, output_scale, output_zero_point)


def rsqrt(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.rsqrt", x, scale, zero_point, output_scale, output_zero_point)


def exp(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.exp", x, scale, zero_point, output_scale, output_zero_point)


def erf(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.erf", x, scale, zero_point, output_scale, output_zero_point)


def sigmoid(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.sigmoid", x, scale, zero_point, output_scale, output_zero_point)


def hardswish(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.hardswish", x, scale, zero_point, output_scale, output_zero_point)


def tanh(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.tanh", x, scale, zero_point, output_scale, output_zero_point)


def log(x, scale, zero_point, output_scale, output_zero_point) -> Call:
    return _unary("qnn.log", x, scale, zero_point, output_scale, output_zero_point)


def abs(x, scale, zero_point, output_scale, output_zero_point) -> Call:  # noqa: A001 (the reference's name)
    return _unary("qnn.abs", x, scale, zero_point, output_scale, output_zero_point)


def batch_matmul(x: Expr, y: Expr, x_zero_point, y_zero_point, x_scale, y_scale, out_dtype="int32") -> Call:
    """``qnn.batch_matmul`` (src/relay/qnn/op/batch_matmul.cc:40-97): [B, M, K] x [B', N, K] (transpose_b,
    B == B' or one of them 1) -> int32 [max(B, B'), M, N]; scalar zero points and scales."""
    if str(np.dtype(out_dtype)) != "int32":
        raise TypeError("qnn.batch_matmul: out_dtype must be int32 (QnnBatchMatmulRel)")
    for e in (x, y):
        if e.dtype not in ("int8", "uint8"):
            raise TypeError(f"qnn.batch_matmul: int8 or uint8 operands expected, got {e.dtype}")
        if len(e.shape) != 3:
            raise TypeError(f"qnn.batch_matmul: rank-3 operands expected, got {e.shape}")
    (bx, m, k), (by, n, k2) = x.shape, y.shape
    if k != k2 or not (bx == by or bx == 1 or by == 1):
        raise TypeError(f"qnn.batch_matmul: {x.shape} x {y.shape}^T")
    args = [x, y, _c(x_zero_point, "int32"), _c(y_zero_point, "int32"), _c(x_scale, "float32"),
            _c(y_scale, "float32")]
    for p in args[2:]:
        if p.checked_type.shape != ():
            raise TypeError("qnn.batch_matmul: zero points and scales must be scalars")
    return Call("qnn.batch_matmul", args, {"transpose_a": False, "transpose_b": True, "out_dtype": "int32"},
                TensorType((max(bx, by), m, n), "int32"))


TRANSPOSE_KERNEL_LAYOUTS = ("IOHW", "OIHW", "HWOI", "HWIO", "OHWI")


def conv2d_transpose(data: Expr, weight: Expr, input_zero_point, kernel_zero_point, input_scale, kernel_scale,
                     strides=(1, 1), padding=(0, 0), dilation=(1, 1), groups: int = 1, channels=None,
                     kernel_size=None, data_layout="NCHW", kernel_layout="IOHW", out_layout="",
                     output_padding=(0, 0), out_dtype="int32") -> Call:
    """``qnn.conv2d_transpose`` (src/relay/qnn/op/convolution_transpose.cc:42-150; Conv2DTransposeRel):
    NCHW / NHWC data; the kernel's 'I' axis is the data's channels, 'O' the output channels per group;
    output in the data layout, (H - 1) * stride + KH - pad_top - pad_bottom + output_padding rows."""
    if data_layout not in ("NCHW", "NHWC") or kernel_layout not in TRANSPOSE_KERNEL_LAYOUTS:
        raise NotImplementedError(f"qnn.conv2d_transpose: data layout {data_layout} / kernel layout {kernel_layout}")
    if out_layout not in ("", data_layout):
        raise NotImplementedError("qnn.conv2d_transpose: out_layout must be the data layout")
    if str(np.dtype(out_dtype)) != "int32":
        raise NotImplementedError("qnn.conv2d_transpose: out_dtype int32 (int16 is not implemented)")
    for e in (data, weight):
        if e.dtype not in ("int8", "uint8"):
            raise TypeError(f"qnn.conv2d_transpose: int8 or uint8 operands expected, got {e.dtype}")
    if tuple(_tuple2(dilation)) != (1, 1):
        raise NotImplementedError("qnn.conv2d_transpose: dilation must be 1 (topi conv2d_transpose_nchw)")
    if data_layout == "NCHW":
        n, c, h, w = data.shape
    else:
        n, h, w, c = data.shape
    ks = dict(zip(kernel_layout, weight.shape))
    ci, og, kh, kw = ks["I"], ks["O"], ks["H"], ks["W"]
    if ci != c or c % groups:
        raise TypeError(f"qnn.conv2d_transpose: kernel {weight.shape} ({kernel_layout}) for {c} channels, "
                        f"groups={groups}")
    if kernel_size is not None and tuple(_tuple2(kernel_size)) != (kh, kw):
        raise TypeError("qnn.conv2d_transpose: kernel_size does not match the kernel shape")
    sh, sw = _tuple2(strides)
    pt, pl, pb, pr = get_pad_tuple2d(padding)
    oph, opw = _tuple2(output_padding)
    if oph >= sh or opw >= sw:
        raise TypeError("qnn.conv2d_transpose: output_padding must be smaller than the stride")
    oh = (h - 1) * sh + kh - pt - pb + oph
    ow = (w - 1) * sw + kw - pl - pr + opw
    o = og * groups
    args = [data, weight, _c(input_zero_point, "int32"), _c(kernel_zero_point, "int32"), _c(input_scale, "float32"),
            _c(kernel_scale, "float32")]
    _scalar_param(args[2], "qnn.conv2d_transpose input_zero_point")
    _scalar_param(args[4], "qnn.conv2d_transpose input_scale")
    attrs = {"strides": (sh, sw), "padding": (pt, pl, pb, pr), "dilation": (1, 1), "groups": int(groups),
             "channels": int(channels) if channels is not None else o, "kernel_size": (kh, kw),
             "data_layout": data_layout, "kernel_layout": kernel_layout, "output_padding": (oph, opw),
             "out_dtype": "int32"}
    shape = (n, o, oh, ow) if data_layout == "NCHW" else (n, oh, ow, o)
    return Call("qnn.conv2d_transpose", args, attrs, TensorType(shape, "int32"))

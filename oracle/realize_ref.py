"""Restatement of the ops a ``relay.quantize``-realized graph runs — TEST INFRASTRUCTURE ONLY.

Integer ops follow the reference bit for bit:
  * ``nn.conv2d`` / ``nn.dense`` int8 x int8 -> int32 (realize.cc:147-174, 207-235): the QNN
    contraction with zero points 0 (qnn_ref.qnn_conv2d / qnn_dense);
  * ``right_shift`` / ``left_shift`` / ``add`` / ``multiply`` on int32 (topi broadcast ops, int32
    wrap-around; right shift is arithmetic);
  * ``fixed_point_multiply`` (topi/math.py:644-673 -> intrin_rule.cc:197-250), the int32 result
    of q_multiply_shift stored in the operand type;
  * ``round`` = llvm.round (halves away from zero); float -> int ``cast`` truncates.
Float ops (the unquantized first conv, the dequantize, the classifier) are restated in a FIXED
summation order: each output accumulates in float32 from 0 over (c, r, s) / k / (h, w) in
row-major order, one rounding per multiply and per add, no fused multiply-add.  The device
kernels use the same order, so parity with this restatement is bit-exact; against the
reference's LLVM build (whose vectorised reduction order is not fixed by Relay) float records
are parity-unpinned at the bit level.
"""
from __future__ import annotations

import numpy as np

from . import qnn_ref as ref

f32 = np.float32


def round_away(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x)
    t = np.trunc(x)
    return (t + np.where(np.abs(x - t) >= 0.5, np.sign(x), 0)).astype(x.dtype)


def _wrap(v: np.ndarray, dtype) -> np.ndarray:
    dt = np.dtype(dtype)
    if dt.itemsize == 8:
        return v.astype(dt)
    return ref.cast(v.astype(np.int64), str(dt))


def binary(op: str, a: np.ndarray, b: np.ndarray, dtype: str) -> np.ndarray:
    if np.dtype(dtype).kind == "f":
        return {"add": np.add, "multiply": np.multiply}[op](a.astype(f32), b.astype(f32)).astype(f32)
    a64, b64 = np.asarray(a).astype(np.int64), np.asarray(b).astype(np.int64)
    with np.errstate(over="ignore"):
        r = {"add": lambda: a64 + b64, "multiply": lambda: a64 * b64, "left_shift": lambda: a64 << b64,
             "right_shift": lambda: a64 >> b64}[op]()
    return _wrap(r, dtype)


def cast(x: np.ndarray, dtype: str) -> np.ndarray:
    dt = np.dtype(dtype)
    if dt.kind == "f":
        return x.astype(dt)
    if x.dtype.kind == "f":
        x = np.trunc(x).astype(np.int64)
    return x.astype(dt) if dt.itemsize == 8 else ref.cast(x, str(dt))


def clip(x: np.ndarray, a_min: float, a_max: float) -> np.ndarray:
    if x.dtype.kind == "f":
        return np.minimum(np.maximum(x, x.dtype.type(a_min)), x.dtype.type(a_max)).astype(x.dtype)
    return ref.clip(x, a_min, a_max)


def fixed_point_multiply(x: np.ndarray, multiplier: int, shift: int) -> np.ndarray:
    """relay.fixed_point_multiply → topi fixed_point_multiply (topi/math.py:644-673) →
    tir.q_multiply_shift legalization (intrin_rule.cc:197-250) in x's dtype: the power-of-two
    case (m == 1<<30, :223-237) shifts and rounds in x's own dtype (int64 wraps at 64 bits), the
    general case (QMultiplyShift, :166-195) casts x to int64 (no narrowing) and the result to
    int32."""
    if x.dtype == np.int64:
        u = x.astype(np.uint64)
        if multiplier == (1 << 30):
            e = shift - 1
            if e > 0:
                return (u << np.uint64(e)).astype(np.int64)
            k = -e
            return (u + np.uint64(1 << (k - 1))).astype(np.int64) >> np.int64(k)
        ls, rs = max(shift, 0), max(-shift, 0)
        return ref._q_multiply_shift_general(x, np.int64(multiplier), ls, rs, ls != 0).astype(np.int64)
    return ref.q_multiply_shift(x.astype(np.int64), multiplier, shift).astype(x.dtype)


def conv2d_f32(x: np.ndarray, w: np.ndarray, strides, padding, dilation, groups) -> np.ndarray:
    n, c, h, wd = x.shape
    o, cg, kh, kw = w.shape
    sh, sw = strides
    dh, dw = dilation
    pt, pl, pb, pr = padding
    xp = np.pad(x.astype(f32), ((0, 0), (0, 0), (pt, pb), (pl, pr)))
    oh = (h + pt + pb - dh * (kh - 1) - 1) // sh + 1
    ow = (wd + pl + pr - dw * (kw - 1) - 1) // sw + 1
    og = o // groups
    out = np.zeros((n, o, oh, ow), f32)
    for g in range(groups):
        acc = np.zeros((n, og, oh, ow), f32)
        for ci in range(cg):
            for r in range(kh):
                for s in range(kw):
                    patch = xp[:, g * cg + ci, r * dh: r * dh + sh * (oh - 1) + 1: sh,
                               s * dw: s * dw + sw * (ow - 1) + 1: sw]
                    prod = (patch[:, None] * w[g * og:(g + 1) * og, ci, r, s].astype(f32)[None, :, None, None])
                    acc = (acc + prod.astype(f32)).astype(f32)
        out[:, g * og:(g + 1) * og] = acc
    return out


def dense_f32(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    acc = np.zeros((x.shape[0], w.shape[0]), f32)
    for k in range(x.shape[1]):
        acc = (acc + (x[:, k:k + 1].astype(f32) * w[:, k].astype(f32)[None, :]).astype(f32)).astype(f32)
    return acc


def max_pool2d_f32(x, pool_size, strides, padding, dilation) -> np.ndarray:
    n, c, h, w = x.shape
    kh, kw = pool_size
    sh, sw = strides
    dh, dw = dilation
    pt, pl, pb, pr = padding
    lo = np.finfo(x.dtype).min
    xp = np.pad(x, ((0, 0), (0, 0), (pt, pb), (pl, pr)), constant_values=lo)
    oh = (h + pt + pb - dh * (kh - 1) - 1) // sh + 1
    ow = (w + pl + pr - dw * (kw - 1) - 1) // sw + 1
    out = np.full((n, c, oh, ow), lo, x.dtype)
    for r in range(kh):
        for s in range(kw):
            out = np.maximum(out, xp[:, :, r * dh: r * dh + sh * (oh - 1) + 1: sh, s * dw: s * dw + sw * (ow - 1) + 1: sw])
    return out


def global_avg_pool2d_f32(x: np.ndarray) -> np.ndarray:
    n, c, h, w = x.shape
    acc = np.zeros((n, c), f32)
    flat = x.reshape(n, c, h * w).astype(f32)
    for i in range(h * w):
        acc = (acc + flat[:, :, i]).astype(f32)
    return (acc / f32(h * w)).astype(f32).reshape(n, c, 1, 1)


def simulated_quantize(x, dom_scale, clip_min, clip_max) -> np.ndarray:
    """_annotate.py:30-47: round(clip(x / s)) * s in float32."""
    s = f32(dom_scale)
    scaled = (x.astype(f32) / s).astype(f32)
    clipped = np.maximum(np.minimum(scaled, f32(clip_max)), f32(clip_min))
    return (round_away(clipped) * s).astype(f32)


def eval_call(call, args):
    """Evaluate one op of a realized (or float) graph; None if it is not one of these ops."""
    op, a = call.op, call.attrs
    dt = call.dtype
    if op == "nn.conv2d":
        if args[0].dtype.kind == "f":
            return conv2d_f32(args[0], args[1], a["strides"], a["padding"], a["dilation"], a["groups"])
        return ref.qnn_conv2d(args[0], args[1], 0, 0, strides=a["strides"], padding=a["padding"],
                              dilation=a["dilation"], groups=a["groups"])
    if op == "nn.dense":
        if args[0].dtype.kind == "f":
            return dense_f32(args[0], args[1])
        return ref.qnn_dense(args[0], args[1], 0, 0)
    if op in ("add", "multiply", "left_shift", "right_shift"):
        return binary(op, args[0], args[1], dt)
    if op == "round":
        return round_away(args[0])
    if op == "fixed_point_multiply":
        return fixed_point_multiply(args[0], a["multiplier"], a["shift"])
    if op in ("annotation.stop_fusion",):
        return args[0]
    if op == "annotation.cast_hint":
        return args[0]
    if op == "relay.op.annotation.simulated_quantize":
        return simulated_quantize(args[0], args[1], args[2], args[3])
    if args and not op.startswith("qnn.") and np.asarray(args[0]).dtype.kind == "f":
        x = args[0]
        if op == "clip":
            return clip(x, a["a_min"], a["a_max"])
        if op == "nn.bias_add":
            ax = a["axis"] if a["axis"] >= 0 else x.ndim + a["axis"]
            return binary("add", x, ref.expand_to_axis(args[1], x.ndim, ax), dt)
        if op == "nn.relu":
            return np.maximum(x, f32(0)).astype(x.dtype)
        if op == "cast":
            return cast(x, a["dtype"])
        if op == "nn.max_pool2d":
            return max_pool2d_f32(x, a["pool_size"], a["strides"], a["padding"], a["dilation"])
        if op == "nn.global_avg_pool2d":
            return global_avg_pool2d_f32(x)
    if op == "cast":
        return cast(args[0], a["dtype"])
    return None


def minimize_kl(hist, edges, num_bins: int, num_quantized_bins: int) -> float:
    """MinimizeKL (src/relay/quantize/calibrate.cc:35-146) in float32 scalar arithmetic, same
    operation order — small num_bins only (pure-Python loops)."""
    F = np.float32
    zero, half_q = num_bins // 2, num_quantized_bins // 2
    thr, div = [], []

    def smooth(p, eps=F(0.0001)):
        zeros = sum(1 for v in p if v == 0)
        nonz = len(p) - zeros
        if nonz == 0:
            return None
        eps1 = F(eps * F(zeros) / F(nonz))
        if eps1 >= 1:
            return None
        return [F(v + F(eps * F(v == 0)) - F(eps1 * F(v != 0))) for v in p]

    for i in range(half_q, zero + 1):
        lo, hi = zero - i, zero + i + 1
        thr.append(F(edges[hi]))
        ln = hi - lo
        win = [0] * ln
        p = [F(0)] * ln
        for j in range(num_bins):
            if j <= lo:
                p[0] = F(p[0] + F(hist[j]))
            elif j >= hi:
                p[-1] = F(p[-1] + F(hist[j]))
            else:
                win[j - lo] = int(hist[j])
                p[j - lo] = F(hist[j])
        per = ln // num_quantized_bins
        merged = [F(sum(win[j * per:(j + 1) * per])) for j in range(num_quantized_bins)]
        merged[-1] = F(merged[-1] + F(sum(win[num_quantized_bins * per:])))
        q = [F(0)] * ln
        for j in range(num_quantized_bins):
            a, b = j * per, (ln if j == num_quantized_bins - 1 else (j + 1) * per)
            nz = sum(1 for k in range(a, b) if win[k] != 0)
            if nz:
                for k in range(a, b):
                    if p[k] != 0:
                        q[k] = F(merged[j] / F(nz))
        p, q = smooth(p), smooth(q)
        if q is None:
            div.append(F(np.inf))
            continue
        p = p or []
        ps, qs = F(0), F(0)
        for v in p:
            ps = F(ps + v)
        for v in q:
            qs = F(qs + v)
        d = F(0)
        for k in range(len(p)):
            pk, qk = F(p[k] / ps), F(q[k] / qs)
            if pk != 0 and qk != 0:
                d = F(d + F(pk * F(np.log(F(pk / qk)))))
        div.append(d)
    return float(thr[int(np.argmin(div))])

"""CPU restatement of the reference's tachikoma BYOC composites (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module;
the product path (tachikoma_amd/) never does.

What it restates
  * ``LegalizeQnnOpForTachikoma`` (python/tvm/relay/op/contrib/tachikoma.py:1122-1306): the
    QNN chain  qnn.conv2d|qnn.dense -> [add bias] -> qnn.requantize(int32) -> clip -> cast
    [-> qnn.add(., sum_src) -> clip]  becomes an int32 contraction with zero zero points and
    float32 post-ops whose constants are folded in float32, in the expression order of
    tachikoma.py:1239-1253 (FoldConstant evaluates the same float32 Relay arithmetic):
        o_scl   = rq_in_scl / rq_out_scl
        act_scl = sum_lhs_scl / sum_out_scl
        sum_scl = sum_rhs_scl / sum_out_scl
        dst_zp  = f(sum_out_zp) - f(sum_lhs_zp) * sum_lhs_scl / sum_out_scl
                                - f(sum_rhs_zp) * sum_rhs_scl / sum_out_scl
        bias    = f(bias) - f(src_zp * sum_k W[oc, k]) - f(rq_in_zp) + f(rq_out_zp) * rq_out_scl / rq_in_scl
  * the runtime's post-op chain (src/runtime/contrib/tachikoma/tachikoma_json_runtime.cc:142-185,
    oneDNN 2.x attributes): output scales on (acc + bias), eltwise clip(0, 255) with scale
    act_scl (the legalized graph's clip, tachikoma.py:1273), sum post-op (sum_scl * the
    destination's previous value, i.e. the sum source), linear eltwise (+ dst_zp), then the
    conversion to the 8-bit destination (round half to even, saturate).

Parity pinning: oneDNN is not vendored in the reference (cmake/modules/contrib/Tachikoma.cmake
finds a system library) and is absent here, so bit-level parity with the reference runtime is
UNPINNED.  The reference's own tests pin the composites to +-1 quantum against TVM's QNN
lowering (tests/python/contrib/test_tachikoma.py:1615-1616, 1761-1762); tests/
test_tachikoma_byoc.py asserts exactly that bound against oracle/qnn_ref.py, and bit-exactness
of the HIP kernel against this module's fixed evaluation order (no fused multiply-add).
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def legalize_constants(w: np.ndarray, bias, src_zp: int, rq_in_scl, rq_in_zp: int, rq_out_scl, rq_out_zp: int,
                       sum_params=None):
    """Float32 constants of the legalized composite (tachikoma.py:1239-1253).

    w: int8 weight with the output channel first (OIHW or [units, K]).  sum_params: None or
    (lhs_scl, lhs_zp, rhs_scl, rhs_zp, out_scl, out_zp) of the qnn.add.
    Returns dict(bias [O], o_scl [O] or scalar, act_scl, sum_scl, dst_zp), all float32."""
    o = w.shape[0]
    rq_in_scl = np.asarray(rq_in_scl, dtype=f32)
    rq_out_scl = f32(rq_out_scl)
    if sum_params is None:  # tachikoma.py:1221-1227 defaults
        lhs_scl, lhs_zp, rhs_scl, rhs_zp, out_scl, out_zp = f32(1.0), 0, f32(0.0), 0, f32(1.0), 0
    else:
        lhs_scl, lhs_zp, rhs_scl, rhs_zp, out_scl, out_zp = sum_params
        lhs_scl, rhs_scl, out_scl = f32(lhs_scl), f32(rhs_scl), f32(out_scl)
    o_scl = (rq_in_scl / rq_out_scl).astype(f32)
    act_scl = f32(lhs_scl / out_scl)
    sum_scl = f32(rhs_scl / out_scl)
    dst_zp = f32(f32(f32(out_zp) - f32(f32(lhs_zp) * lhs_scl) / out_scl) - f32(f32(rhs_zp) * rhs_scl) / out_scl)
    # fake_op (tachikoma.py:1280-1288): zp * the kernel summed over every axis but O
    wsum = w.reshape(o, -1).astype(np.int64).sum(axis=1).astype(np.int32)
    fake = (np.int32(src_zp) * wsum).astype(np.int32)
    b = np.zeros(o, np.int32) if bias is None else np.asarray(bias, np.int32).reshape(o)
    t = (b.astype(f32) - fake.astype(f32)).astype(f32)
    t = (t - f32(rq_in_zp)).astype(f32)
    u = (f32(f32(rq_out_zp) * rq_out_scl) / rq_in_scl).astype(f32)
    bias_f = (t + u).astype(f32)
    return {"bias": bias_f, "o_scl": o_scl, "act_scl": act_scl, "sum_scl": sum_scl, "dst_zp": dst_zp}


def postops(acc: np.ndarray, consts, out_dtype: str, sum_src=None, channel_axis: int = 1,
            clip=(0.0, 255.0)) -> np.ndarray:
    """Post-op chain on the int32 contraction ``acc`` (zero zero points), in float32:
    t = (f(acc) + bias) * o_scl; t = clip(t) * act_scl; t = sum_scl * f(sum_src) + t;
    t = t + dst_zp; round half to even; saturate to out_dtype."""
    shape = [1] * acc.ndim
    shape[channel_axis] = acc.shape[channel_axis]
    bias = np.asarray(consts["bias"], f32).reshape(shape)
    o_scl = np.asarray(consts["o_scl"], f32)
    o_scl = o_scl.reshape(shape) if o_scl.ndim else o_scl
    t = (acc.astype(f32) + bias).astype(f32)
    t = (t * o_scl).astype(f32)
    t = np.minimum(np.maximum(t, f32(clip[0])), f32(clip[1])).astype(f32)
    t = (t * f32(consts["act_scl"])).astype(f32)
    if sum_src is not None:
        t = ((f32(consts["sum_scl"]) * sum_src.astype(f32)).astype(f32) + t).astype(f32)
    t = (t + f32(consts["dst_zp"])).astype(f32)
    info = np.iinfo(np.dtype(out_dtype))
    r = np.rint(t)  # round half to even (the default floating-point rounding mode)
    return np.clip(r, info.min, info.max).astype(out_dtype)

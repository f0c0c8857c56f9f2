"""CPU evaluation of the canonical (post-QNN-lowering) graph, tachikoma_amd/relay/canonical.py:
the integer ops the reference's executor runs after legalization / canonicalization -- int16 data
shifts, int16 x int16 -> int32 contractions, the requantize chain (int32 cast, zero-point
subtract, ``fixed_point_multiply`` / ``fixed_point_multiply_per_axis``, output zero-point add,
clip, cast), qnn.add's RequantizeOrUpcast sums.  Test infrastructure only (the fused-node debug
dump is checked against it).  Each op wraps in its dtype like the reference's TIR."""
import numpy as np

from . import qnn_ref as ref
from . import realize_ref


def _wrap(v, dtype) -> np.ndarray:
    dt = np.dtype(dtype)
    bits = dt.itemsize * 8
    v = np.asarray(v, dtype=np.int64)
    if bits < 64:
        m = 1 << bits
        v = v & (m - 1)
        if dt.kind == "i":
            v = np.where(v >= (m >> 1), v - m, v)
    return v.astype(dt)


def _axis_vec(vec, ndim: int, axis: int) -> np.ndarray:
    axis = axis if axis >= 0 else ndim + axis
    shape = [1] * ndim
    shape[axis] = -1
    return np.asarray(vec).reshape(shape)


def _qms_general(x: np.ndarray, m: np.ndarray, s: np.ndarray) -> np.ndarray:
    """q_multiply_shift general form (intrin_rule.cc:166-195), elementwise m / s: per-axis always
    takes it, also for m == 2^30 (:252-267)."""
    x = np.asarray(x, np.int64)
    ls = np.maximum(s, 0).astype(np.int64)
    rs = np.maximum(-s, 0).astype(np.int64)
    with np.errstate(over="ignore"):
        y = (x.astype(np.uint64) << ls.astype(np.uint64)).astype(np.int64)
        y = (y.astype(np.uint64) * m.astype(np.int64).astype(np.uint64)).astype(np.int64)
        total = 31 + rs
        y = (y.astype(np.uint64) + (np.uint64(1) << (total - 1).astype(np.uint64))).astype(np.int64)
        y = y >> total
    return _wrap(y, "int32")


def eval_op(op, args):
    a = op.attrs
    dt = op.out.dtype
    x = args[0] if args else None
    if op.op == "cast":
        return _wrap(x, dt)
    if op.op == "subtract":
        if "vector" in op.consts:
            return _wrap(x.astype(np.int64) - _axis_vec(op.consts["vector"], x.ndim, a["axis"]), dt)
        return _wrap(x.astype(np.int64) - a["scalar"], dt)
    if op.op == "add" and len(args) == 2 and dt == "int64":
        with np.errstate(over="ignore"):
            return (np.asarray(x, np.int64).astype(np.uint64) + np.asarray(args[1], np.int64).astype(np.uint64)
                    ).astype(np.int64)
    if op.op == "add":
        if "scalar" in a:
            return _wrap(x.astype(np.int64) + a["scalar"], dt)
        y = args[1].astype(np.int64)
        if "axis" in a and y.shape != x.shape:
            y = _axis_vec(y.reshape(-1), x.ndim, a["axis"])
        return _wrap(x.astype(np.int64) + y, dt)
    if op.op == "fixed_point_multiply":
        return realize_ref.fixed_point_multiply(x, a["multiplier"], a["shift"])
    if op.op == "fixed_point_multiply_per_axis":
        m = _axis_vec(op.consts["multipliers"], x.ndim, a["axis"])
        s = _axis_vec(op.consts["shifts"], x.ndim, a["axis"])
        return _qms_general(x, np.broadcast_to(m, x.shape), np.broadcast_to(s, x.shape))
    if op.op in ("left_shift", "right_shift", "multiply"):
        # int64 steps of FixedPointMultiplyToNearest (src/relay/qnn/utils.cc:59-216), wrapping
        v = np.int64(a["scalar"]) if "scalar" in a else _axis_vec(op.consts["vector"], x.ndim, a["axis"])
        x64 = np.asarray(x, np.int64)
        with np.errstate(over="ignore"):
            if op.op == "left_shift":
                y = (x64.astype(np.uint64) << np.asarray(v).astype(np.uint64)).astype(np.int64)
            elif op.op == "right_shift":
                y = x64 >> np.asarray(v).astype(np.int64)
            else:
                y = (x64.astype(np.uint64) * np.asarray(v).astype(np.int64).astype(np.uint64)).astype(np.int64)
        return _wrap(y, dt)
    if op.op == "greater_equal":
        return np.asarray(x) >= a["scalar"]
    if op.op == "where":
        pos, neg = op.consts["pos"], op.consts["neg"]
        if "axis" in a:
            pos, neg = _axis_vec(pos, x.ndim, a["axis"]), _axis_vec(neg, x.ndim, a["axis"])
        else:
            pos, neg = pos.reshape(()), neg.reshape(())
        return np.where(x, pos, neg).astype(dt)
    if op.op == "clip":
        return np.clip(x, a["a_min"], a["a_max"]).astype(x.dtype)
    if op.op == "nn.relu":
        return np.maximum(x, 0).astype(x.dtype)
    if op.op in ("nn.conv2d", "nn.dense"):
        zw = op.consts.get("kernel_zero_points", op.consts["kernel_zero_point"])
        if op.op == "nn.conv2d":
            return ref.qnn_conv2d(x, args[1], 0, zw, strides=a["strides"], padding=a["padding"],
                                  dilation=a["dilation"], groups=a["groups"])
        return ref.qnn_dense(x, args[1], 0, zw)
    if op.op == "nn.max_pool2d":
        return ref.max_pool2d(x, a["pool_size"], a["strides"], a["padding"], a["dilation"])
    if op.op == "nn.avg_pool2d":
        return ref.avg_pool2d(x, a["pool_size"], a["strides"], a["padding"], a["dilation"],
                              a.get("count_include_pad", False))
    if op.op == "nn.global_avg_pool2d":
        return ref.global_avg_pool2d(x)
    if op.op in ("nn.batch_flatten", "reshape"):
        return np.asarray(x).reshape(op.out.shape)
    raise NotImplementedError(op.op)


def evaluate(canon, values):
    """{canonical tensor: value} for every op of ``canon``, given the plan's input / param values."""
    vals = dict(values)
    for op in canon.ops:
        vals[op.name] = eval_op(op, [vals[x] for x in op.inputs])
    return vals

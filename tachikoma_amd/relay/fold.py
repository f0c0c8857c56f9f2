"""Host-side constant folding (``relay.transform.FoldConstant`` for the ops the quantizer
leaves on constants): a call whose arguments are all constants is evaluated on the host at
build time, like the reference's FoldConstant evaluates them with its CPU executor
(src/relay/transforms/fold_constant.cc).  Compile-time only: nothing here runs per sample.
"""
from __future__ import annotations

import math
from typing import Callable, Dict

import numpy as np

from .expr import Call, Constant, Expr, Function, IRModule, Var, post_order


def round_away(x: np.ndarray) -> np.ndarray:
    """``round`` = llvm.round: halves away from zero, exact in float32."""
    x = np.asarray(x)
    t = np.trunc(x)
    frac = np.abs(x - t)  # exact: x and trunc(x) share the exponent range
    return (t + np.where(frac >= 0.5, np.sign(x), 0)).astype(x.dtype)


def _int_wrap(v: np.ndarray, dtype) -> np.ndarray:
    bits = np.dtype(dtype).itemsize * 8
    v = np.asarray(v, np.int64) if bits < 64 else np.asarray(v).astype(np.int64)
    if bits < 64:
        m = 1 << bits
        v = ((v + (m >> 1)) & (m - 1)) - (m >> 1) if np.issubdtype(np.dtype(dtype), np.signedinteger) else v & (m - 1)
    return v.astype(dtype)


def _cast(x: np.ndarray, dtype: str) -> np.ndarray:
    dt = np.dtype(dtype)
    if dt.kind == "f":
        return x.astype(dt)
    if x.dtype.kind == "f":  # fptosi truncates toward zero
        return _int_wrap(np.trunc(x).astype(np.int64), dt)
    return _int_wrap(x.astype(np.int64), dt)


def _clip(x: np.ndarray, lo: float, hi: float) -> np.ndarray:
    if x.dtype.kind == "f":
        return np.minimum(np.maximum(x, x.dtype.type(lo)), x.dtype.type(hi)).astype(x.dtype)
    info = np.iinfo(x.dtype)
    lo_i = max(int(math.trunc(lo)) if math.isfinite(lo) else int(info.min), int(info.min))
    hi_i = min(int(math.trunc(hi)) if math.isfinite(hi) else int(info.max), int(info.max))
    return np.minimum(np.maximum(x, lo_i), hi_i).astype(x.dtype)


def _binary(op: str, a: np.ndarray, b: np.ndarray, dtype: str) -> np.ndarray:
    if np.dtype(dtype).kind == "f":
        r = {"add": np.add, "multiply": np.multiply, "subtract": np.subtract, "divide": np.divide}[op](a, b)
        return r.astype(dtype)
    a64, b64 = a.astype(np.int64), b.astype(np.int64)
    if op == "add":
        r = a64 + b64
    elif op == "multiply":
        r = a64 * b64
    elif op == "subtract":
        r = a64 - b64
    elif op == "left_shift":
        r = a64 << b64
    elif op == "right_shift":
        r = a64 >> b64
    else:
        raise NotImplementedError(op)
    return _int_wrap(r, dtype)


def eval_const_call(call: Call, args) -> np.ndarray:
    op, a = call.op, call.attrs
    if op in ("add", "multiply", "subtract", "left_shift", "right_shift") or (op == "divide" and call.dtype == "float32"):
        return _binary(op, args[0], args[1], call.dtype)
    if op == "sqrt" and call.dtype == "float32":  # llvm.sqrt.f32: correctly rounded, as np.sqrt
        return np.sqrt(args[0]).astype(np.float32)
    if op == "negative":
        return (-args[0]).astype(args[0].dtype) if call.dtype == "float32" else _int_wrap(-args[0].astype(np.int64), call.dtype)
    if op == "round":
        return round_away(args[0])
    if op == "clip":
        return _clip(args[0], a["a_min"], a["a_max"])
    if op in ("cast", "annotation.cast_hint"):
        return _cast(args[0], call.dtype)
    if op in ("annotation.stop_fusion", "nn.batch_flatten", "reshape"):
        return args[0].reshape(call.shape)
    if op == "expand_dims":
        return args[0].reshape(call.shape)
    raise NotImplementedError(f"constant folding of {op}")


def rebuild(body: Expr, fn: Callable[[Call, list], Expr]) -> Expr:
    """Post-order mutator: ``fn(call, new_args)`` returns the replacement of each call (tuples are
    rebuilt around rewritten fields)."""
    from .expr import Tuple
    new: Dict[int, Expr] = {}
    for n in post_order(body):
        if isinstance(n, Call):
            args = [new.get(id(x), x) for x in n.args]
            new[id(n)] = fn(n, args)
        elif isinstance(n, Tuple):
            fields = [new.get(id(x), x) for x in n.fields]
            if any(x is not y for x, y in zip(fields, n.fields)):
                new[id(n)] = Tuple(fields)
    return new.get(id(body), body)


def fold_constant(mod) -> IRModule:
    func = mod["main"] if isinstance(mod, IRModule) else IRModule.from_expr(mod)["main"]

    def fold(call: Call, args):
        if args and all(isinstance(x, Constant) for x in args):
            try:
                return Constant(eval_const_call(call, [x.data for x in args]))
            except NotImplementedError:
                pass
        if all(x is y for x, y in zip(args, call.args)):
            return call
        return Call(call.op, args, call.attrs, call.checked_type)

    body = rebuild(func.body, fold)
    return IRModule(Function([p for p in func.params if isinstance(p, Var)], body))

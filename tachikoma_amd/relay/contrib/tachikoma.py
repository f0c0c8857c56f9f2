"""The reference's tachikoma BYOC composites, offloaded to the MI355X engine.

Reference: python/tvm/relay/op/contrib/tachikoma.py
  * ``make_qnn_conv2d_pattern`` / ``make_qnn_dense_pattern`` (:356-415) and ``pattern_table``
    (:418-458): the composites ``tachikoma.qnn.conv2d`` / ``tachikoma.qnn.dense``;
  * ``LegalizeQnnOpForTachikoma`` (:1122-1306) + ``legalize_qnn_for_tachikoma`` (:1308-1323):
    the QNN chain
        qnn.conv2d|qnn.dense(src, wgh, src_zp, 0, ...) -> [add bias] -> qnn.requantize -> clip
        -> cast [-> qnn.add(cast, sum_src, ...) -> clip]
    becomes an int32 contraction with zero zero points plus float32 post-ops
        ((acc + bias) * o_scl -> clip(0, 255) * act_scl [+ sum_scl * sum_src] + dst_zp -> cast)
    with the constants folded in float32 (FoldConstant);
  * the runtime executes the composite as one oneDNN primitive with post-ops
    (src/runtime/contrib/tachikoma/tachikoma_json_runtime.cc:142-185, 292-502).

Here ``partition_for_tachikoma`` rewrites a graph of this package's IR so that every matched
chain is ONE call of the composite op (the reference's composite function: one graph-executor
node, hence one trace record), carrying the folded constants.  ``relay.build`` lowers it to a
contraction kernel writing an untraced int32 buffer plus ``tk_tachikoma_postops``
(include/tachikoma.h).  Parity: the reference pins the composites to +-1 quantum against the
QNN path (tests/python/contrib/test_tachikoma.py:1615-1616, 1761-1762).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from ..expr import Call, Constant, Expr, Function, IRModule, TensorType, Var, post_order

f32 = np.float32

COMPOSITES = ("tachikoma.qnn.conv2d", "tachikoma.qnn.dense")


def pattern_table():
    """Composite names and the op chain each matches (tachikoma.py:356-458, QNN entries)."""
    chain = ["cast", "add (optional bias)", "multiply o_scl", "clip", "multiply act_scl (optional)",
             "add sum_scl * cast(sum_src) (optional)", "add dst_zp (optional)", "cast"]
    return [("tachikoma.qnn.conv2d", ["qnn.conv2d"] + chain), ("tachikoma.qnn.dense", ["qnn.dense"] + chain)]


def _const(e: Expr, what: str) -> np.ndarray:
    if not isinstance(e, Constant):
        raise ValueError(f"{what} must be a constant")
    return e.data


def _value(e: Expr, params: Dict[str, np.ndarray], what: str) -> np.ndarray:
    if isinstance(e, Constant):
        return e.data
    if isinstance(e, Var) and e.name_hint in params:
        return np.asarray(params[e.name_hint])
    raise ValueError(f"{what} must be a constant or a bound param")


def _match(root: Call, consumers: Dict[int, int]) -> Optional[dict]:
    """Match the legalization pattern (tachikoma.py:1173-1193) rooted at ``root``: the sum form
    clip(qnn.add(cast(...), sum_src)) or the plain form cast(clip(requantize(...)))."""
    def single(e):
        return isinstance(e, Call) and consumers.get(id(e), 0) == 1

    m = {}
    node = root
    if root.op == "clip" and isinstance(root.args[0], Call) and root.args[0].op == "qnn.add":
        qadd = root.args[0]
        if not single(qadd) or not isinstance(qadd.args[0], Call) or qadd.args[0].op != "cast":
            return None
        m["sum_add"], m["sum_src"] = qadd, qadd.args[1]
        node = qadd.args[0]
    if not (isinstance(node, Call) and node.op == "cast"):
        return None
    cast = node
    if "sum_add" in m and not single(cast):
        return None
    cl = cast.args[0]
    if not (single(cl) and cl.op == "clip"):
        return None
    rq = cl.args[0]
    if not (single(rq) and rq.op == "qnn.requantize"):
        return None
    x = rq.args[0]
    bias = None
    if single(x) and x.op in ("add", "nn.bias_add"):
        bias = x.args[1]
        x = x.args[0]
    if not (single(x) and x.op in ("qnn.conv2d", "qnn.dense")):
        return None
    zw = x.args[3]
    if not (isinstance(zw, Constant) and zw.data.ndim == 0 and int(zw.data) == 0):
        return None  # the pattern requires a zero kernel zero point (tachikoma.py:1159)
    m.update(root=root, cast=cast, rq=rq, bias=bias, contraction=x)
    return m


def _legalize(m: dict, params: Dict[str, np.ndarray]) -> dict:
    """Folded float32 constants, in the expression order of tachikoma.py:1239-1253."""
    x, rq = m["contraction"], m["rq"]
    w = _value(x.args[1], params, "tachikoma composite weight")
    src_zp = int(_const(x.args[2], "input zero point"))
    rq_in_scl = np.asarray(_const(rq.args[1], "requantize input scale"), f32)
    rq_in_zp = _const(rq.args[2], "requantize input zero point")
    rq_out_scl = f32(_const(rq.args[3], "requantize output scale"))
    rq_out_zp = _const(rq.args[4], "requantize output zero point")
    if np.ndim(rq_in_zp) or np.ndim(rq_out_zp):
        raise ValueError("tachikoma composite: per-channel requantize zero points are not supported")
    if "sum_add" in m:
        c = [_const(m["sum_add"].args[i], "qnn.add parameter") for i in range(2, 8)]
        if any(np.ndim(v) for v in c):
            raise ValueError("tachikoma composite: per-channel qnn.add parameters are not supported")
        lhs_scl, lhs_zp, rhs_scl, rhs_zp, out_scl, out_zp = f32(c[0]), int(c[1]), f32(c[2]), int(c[3]), f32(c[4]), int(c[5])
    else:  # tachikoma.py:1221-1227
        lhs_scl, lhs_zp, rhs_scl, rhs_zp, out_scl, out_zp = f32(1.0), 0, f32(0.0), 0, f32(1.0), 0
    o = w.shape[0]
    o_scl = (rq_in_scl / rq_out_scl).astype(f32)
    act_scl = f32(lhs_scl / out_scl)
    sum_scl = f32(rhs_scl / out_scl)
    dst_zp = f32(f32(f32(out_zp) - f32(f32(lhs_zp) * lhs_scl) / out_scl) - f32(f32(rhs_zp) * rhs_scl) / out_scl)
    # fake_op: src_zp * the kernel summed over every axis but O (tachikoma.py:1280-1288), in int32
    wsum = w.reshape(o, -1).astype(np.int64).sum(axis=1)
    fake = (np.int64(src_zp) * wsum).astype(np.int32)
    if m["bias"] is None:
        b = np.zeros(o, np.int32)
    else:
        b = np.asarray(_value(m["bias"], params, "tachikoma composite bias"), np.int32).reshape(o)
    t = (b.astype(f32) - fake.astype(f32)).astype(f32)
    t = (t - f32(int(rq_in_zp))).astype(f32)
    bias_f = (t + (f32(f32(int(rq_out_zp)) * rq_out_scl) / rq_in_scl).astype(f32)).astype(f32)
    return {"bias": bias_f, "o_scl": o_scl, "act_scl": act_scl, "sum_scl": sum_scl, "dst_zp": dst_zp,
            "clip": (0.0, 255.0)}  # the legalized graph clips to [0, 255] (tachikoma.py:1273)


def _composite(m: dict, params) -> Call:
    x = m["contraction"]
    po = _legalize(m, params)
    final = m["root"].dtype
    name = "tachikoma.qnn.conv2d" if x.op == "qnn.conv2d" else "tachikoma.qnn.dense"
    attrs = {k: v for k, v in x.attrs.items() if k != "out_dtype"}
    attrs.update(postops=po, out_dtype=final)
    args: List[Expr] = [x.args[0], x.args[1]]
    if "sum_src" in m:
        args.append(m["sum_src"])
    return Call(name, args, attrs, TensorType(m["root"].shape, final))


def partition_for_tachikoma(mod, params: Optional[Dict[str, np.ndarray]] = None) -> IRModule:
    """``partition_for_tachikoma`` (tachikoma.py) for the QNN composites: legalize and merge
    every matching chain into one composite call.  Weights and biases must be constants or
    params (their values fold into the composite's constants, as FoldConstant does)."""
    func = mod["main"] if isinstance(mod, IRModule) else IRModule.from_expr(mod)["main"]
    params = {k: np.asarray(v.numpy() if hasattr(v, "numpy") else v) for k, v in (params or {}).items()}
    nodes = post_order(func.body)
    consumers: Dict[int, int] = {}
    for n in nodes:
        for a in getattr(n, "args", []):
            consumers[id(a)] = consumers.get(id(a), 0) + 1
    consumers[id(func.body)] = consumers.get(id(func.body), 0) + 1
    new: Dict[int, Expr] = {}

    def rebuilt(e: Expr) -> Expr:
        return new.get(id(e), e)

    for n in nodes:
        if not isinstance(n, Call):
            continue
        m = _match(n, consumers)
        if m is not None:
            c = _composite(m, params)
            c.args = [rebuilt(a) for a in c.args]
            new[id(n)] = c
            continue
        args = [rebuilt(a) for a in n.args]
        if any(a is not b for a, b in zip(args, n.args)):
            new[id(n)] = Call(n.op, args, n.attrs, n.checked_type)
    return IRModule(Function(func.params, rebuilt(func.body)))


def legalize_qnn_for_tachikoma(mod, params=None) -> IRModule:
    """Alias kept for the reference's entry-point name (legalization and merging happen together
    here: the composite call is the legalized form)."""
    return partition_for_tachikoma(mod, params)

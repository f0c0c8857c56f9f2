"""Graph rewrites the reference runs ahead of quantization and lowering (``relay.transform``):
``SimplifyInference`` (src/relay/transforms/simplify_inference.cc), ``FoldScaleAxis`` in its
backward direction (src/relay/transforms/fold_scale_axis.cc) and ``FoldConstant``
(src/relay/transforms/fold_constant.cc, here ``fold.fold_constant``).

``relay.quantize``'s ``prerequisite_optimize`` (python/tvm/relay/quantize/quantize.py:312-322) runs
SimplifyInference -> FoldConstant -> FoldScaleAxis -> CanonicalizeOps -> FoldConstant, so a float
model with ``nn.batch_norm`` layers reaches the quantizer as convolutions with the batch norm's
scale folded into their weights and its shift left as a constant ``add``.  Host-side, build time
only.  Each pass is a function over an IRModule (or expression) and a pass object with the
reference's constructor name (``SimplifyInference()(mod)``).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from . import op as _op
from .expr import Call, Constant, Expr, Function, IRModule, Var, post_order
from .fold import fold_constant, rebuild

__all__ = ["simplify_inference", "fold_scale_axis", "fold_constant", "SimplifyInference", "FoldScaleAxis",
           "FoldConstant"]


def _func(mod) -> Function:
    return mod["main"] if isinstance(mod, IRModule) else IRModule.from_expr(mod)["main"]


def _module(func: Function, body: Expr) -> IRModule:
    return IRModule(Function([p for p in func.params if isinstance(p, Var)], body))


def _expand_to_axis(v: Expr, ndim: int, axis: int) -> Expr:
    """ExpandBiasToMatchAxis (src/relay/transforms/pattern_utils.h:190-213) for one axis: a [C]
    vector becomes [C, 1, ...] with ndim - axis - 1 trailing unit dimensions."""
    trail = ndim - axis - 1
    if trail <= 0:
        return v
    return _op.reshape(v, (v.shape[0],) + (1,) * trail)


def simplify_inference(mod) -> IRModule:
    """SimplifyInference: every ``nn.batch_norm`` (its normalised output) becomes
    ``add(multiply(data, scale), shift)`` with (BatchNormToInferUnpack, simplify_inference.cc:33-62)
    ``scale = 1 / sqrt(moving_var + epsilon) [* gamma]`` and
    ``shift = -moving_mean * scale [+ beta]``, both expanded along the batch norm's axis.  The
    scale / shift arithmetic stays in the graph as float ops on constants, which FoldConstant then
    evaluates in the data's dtype (float32), as the reference's FoldConstant does."""
    func = _func(mod)

    def rw(call: Call, args):
        if call.op != "nn.batch_norm":
            if all(x is y for x, y in zip(args, call.args)):
                return call
            return Call(call.op, args, call.attrs, call.checked_type)
        data, gamma, beta, mean, var = args
        a = call.attrs
        dt = data.dtype
        eps = Constant(np.asarray(np.float32(a["epsilon"])).astype(dt))
        scale = Call("divide", [Constant(np.asarray(1.0, dt)), Call("sqrt", [_op.add(var, eps)], {}, var.checked_type)],
                     {}, var.checked_type)
        if a["scale"]:
            scale = _op.multiply(scale, gamma)
        shift = _op.multiply(Call("negative", [mean], {}, mean.checked_type), scale)
        if a["center"]:
            shift = _op.add(shift, beta)
        ndim = len(data.shape)
        axis = a["axis"] if a["axis"] >= 0 else a["axis"] + ndim
        out = _op.multiply(data, _expand_to_axis(scale, ndim, axis))
        return _op.add(out, _expand_to_axis(shift, ndim, axis))

    return _module(func, rebuild(func.body, rw))


def _channel_scale(c: Expr, out: Expr) -> Optional[np.ndarray]:
    """The per-output-channel vector of a constant multiplier of ``out`` (NCHW: [C, 1, 1] or
    [1, C, 1, 1]; [N, units] dense: [units] or [1, units]), or None."""
    if not isinstance(c, Constant) or c.data.dtype != np.dtype(out.dtype):
        return None
    shape, d = tuple(out.shape), c.data
    if len(shape) == 4 and d.shape in ((shape[1], 1, 1), (1, shape[1], 1, 1)):
        return d.reshape(-1)
    if len(shape) == 2 and d.shape in ((shape[1],), (1, shape[1])):
        return d.reshape(-1)
    return None


def fold_scale_axis(mod) -> IRModule:
    """FoldScaleAxis, backward direction (fold_scale_axis.cc BackwardFoldScaleAxis): a
    ``multiply`` by a per-output-channel constant is folded into the producer of its data when
    every node on the way has this multiply as its only consumer:

    * ``nn.conv2d(x, W)`` (NCHW / OIHW, groups == 1 or depthwise: output channel o is weight row o)
      -> ``nn.conv2d(x, W * s[o])`` (Conv2DBackwardTransform);
    * ``nn.dense(x, W)`` -> ``nn.dense(x, W * s[:, None])`` (DenseBackwardTransform);
    * ``add(a, b)`` -> ``add(fold(a), fold(b))`` when both sides fold, a constant side (a bias
      [C, 1, 1] / [1, C, 1, 1], or [C] / [1, C] on a dense output) being multiplied by s
      (AddSubBackwardTransform).

    The new weights are ``multiply`` calls on constants that the FoldConstant after this pass
    evaluates (float32 elementwise, like the reference).  The forward direction (a scale on a
    conv's input channels) is not implemented: in the batch-norm graphs of this path the
    scale and shift of a pre-activation batch norm reach the next conv through an ``add`` and a
    ``relu``, which the reference's forward pass does not fold through either."""
    func = _func(mod)
    uses: Dict[int, int] = {}
    for n in post_order(func.body):
        for a in getattr(n, "args", []):
            uses[id(a)] = uses.get(id(a), 0) + 1

    def fold(e: Expr, orig: Expr, s: np.ndarray, ndim: int) -> Optional[Expr]:
        """e: the rewritten node, orig: the node it replaces (use counts are the original graph's),
        ndim: the rank of the tensor ``s`` scales along its channel axis (1)."""
        if isinstance(e, Constant):
            # only a constant that broadcasts onto the channel axis of a rank-``ndim`` output
            # (AddSubBackwardPrep's MatchBroadcastToLeftAxes, fold_scale_axis.cc): a (C,) vector
            # on an NCHW output would broadcast along W instead
            shape, c = tuple(e.data.shape), len(s)
            if e.data.dtype.kind != "f":
                return None
            if ndim == 4 and shape in ((c, 1, 1), (1, c, 1, 1)):
                return _op.multiply(e, Constant(s.reshape(shape)))
            if ndim == 2 and shape in ((c,), (1, c)):
                return _op.multiply(e, Constant(s.reshape(shape)))
            return None
        if not isinstance(e, Call) or uses.get(id(orig), 0) != 1:
            return None
        if e.op == "nn.conv2d" and e.dtype == "float32" and isinstance(e.args[1], Constant):
            w = e.args[1]
            # ConvBackwardPrep folds only into groups == 1 or depthwise convs (fold_scale_axis.cc:
            # 986-987; IsDepthwiseConv, pattern_utils.h:223-229: O == groups and I == 1)
            g = int(e.attrs.get("groups", 1))
            if not (g == 1 or (w.data.shape[0] == g and w.data.shape[1] == 1)):
                return None
            nw = _op.multiply(w, Constant(s.reshape(-1, 1, 1, 1).astype(w.data.dtype)))
            return Call("nn.conv2d", [e.args[0], nw], e.attrs, e.checked_type)
        if e.op == "nn.dense" and e.dtype == "float32" and isinstance(e.args[1], Constant):
            w = e.args[1]
            return Call("nn.dense", [e.args[0], _op.multiply(w, Constant(s.reshape(-1, 1).astype(w.data.dtype)))],
                        e.attrs, e.checked_type)
        if e.op == "add":
            a = fold(e.args[0], orig.args[0], s, len(e.shape))
            b = fold(e.args[1], orig.args[1], s, len(e.shape))
            if a is None or b is None:
                return None
            return _op.add(a, b)
        return None

    def rw(call: Call, args):
        if call.op == "multiply" and call.dtype == "float32":
            s = _channel_scale(args[1], call)
            if s is not None:
                folded = fold(args[0], call.args[0], s, len(call.shape))
                if folded is not None:
                    return folded
        if all(x is y for x, y in zip(args, call.args)):
            return call
        return Call(call.op, args, call.attrs, call.checked_type)

    return _module(func, rebuild(func.body, rw))


class _Pass:
    def __init__(self, fn):
        self.fn = fn

    def __call__(self, mod):
        return self.fn(mod)


def SimplifyInference() -> _Pass:  # noqa: N802  (relay.transform.SimplifyInference)
    return _Pass(simplify_inference)


def FoldScaleAxis() -> _Pass:  # noqa: N802
    return _Pass(fold_scale_axis)


def FoldConstant() -> _Pass:  # noqa: N802
    return _Pass(fold_constant)

"""The quantization passes: partition, annotate, calibrate, realize (+ the driver).

Each pass is a forward rewrite with per-op rules, the way the reference drives them through
``ForwardRewrite`` (src/relay/transforms/forward_rewrite.cc) with temporary expressions that
carry pass state between a producer and its consumers:

* partition  (python/tvm/relay/quantize/_partition.py, src/relay/quantize/partition.cc:40-46):
  ``QPartitionExpr`` -> ``stop_fusion(cast_hint(x, dtype_input))`` where a quantized region ends;
* annotate   (_annotate.py:156-410, annotate.cc:41-90): ``QAnnotateExpr(kind)``, attaching
  ``simulated_quantize(x, dom_scale, clip_min, clip_max, kind)`` to operands;
* calibrate  (_calibrate.py:158-238): binds each simulated_quantize's scale and clip range
  (``global_scale`` for inputs/activations, ``power2`` or ``max`` for weights);
* realize    (realize.cc:45-520): ``QRealizeIntExpr(data, dom_scale, dtype)`` -> integer ops
  (``nn.conv2d`` int8 x int8 -> int32, ``add``, ``left_shift``/``right_shift``,
  ``fixed_point_multiply``, ``clip``, ``cast``), dequantizing (``cast`` + ``multiply``) where a
  float consumer needs the value.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional

import numpy as np

from .. import op as _op
from ..expr import Call, Constant, Expr, Function, IRModule, TensorType, Var, post_order
from ..fold import fold_constant, rebuild
from ..build_module import UnsupportedError
from .qconfig import QAnnotateKind, current_qconfig

SQ = "relay.op.annotation.simulated_quantize"
f32 = np.float32


# ----------------------------------------------------------------------------- rewrite engine

class _Temp:
    """A pass-local temporary (TempExpr): ``realize()`` turns it into a plain expression."""

    def realize(self) -> Expr:
        raise NotImplementedError


def _real(e):
    return e.realize() if isinstance(e, _Temp) else e


def _forward_rewrite(func: Function, rules: Dict[str, Callable], fmulti_ref: Optional[Callable] = None) -> Function:
    """ForwardRewrite: post-order; each call's rule sees the rewritten arguments (temporaries
    included) and returns a replacement or None (then the arguments are realized and the op is
    kept).  ``fmulti_ref`` transforms an argument referenced more than once."""
    body = func.body
    nodes = post_order(body)
    refs: Dict[int, int] = {}
    for n in nodes:
        for a in getattr(n, "args", []):
            refs[id(a)] = refs.get(id(a), 0) + 1
    post: Dict[int, object] = {}
    for n in nodes:
        if not isinstance(n, Call):
            post[id(n)] = n
            continue
        rule = rules.get(n.op)
        args = []
        for a in n.args:
            v = post[id(a)]
            if fmulti_ref is not None and refs.get(id(a), 0) > 1:
                v = fmulti_ref(v)
            args.append(v if rule is not None else _real(v))
        res = rule(n, args) if rule is not None else None
        if res is not None:
            post[id(n)] = res
            continue
        args = [_real(v) for v in args]
        post[id(n)] = n if all(x is y for x, y in zip(args, n.args)) else _forward(n, args)
    out = _real(post[id(body)])
    return Function(_params_of(out, func.params), out)


def _params_of(body: Expr, old: List[Var]) -> List[Var]:
    live = {id(v) for v in post_order(body) if isinstance(v, Var)}
    ps = [v for v in old if id(v) in live]
    seen = {id(v) for v in ps}
    ps += [v for v in post_order(body) if isinstance(v, Var) and id(v) not in seen]
    return ps


def _forward(ref: Call, args: List[Expr], attrs=None) -> Call:
    """Re-create ``ref`` over new arguments, re-inferring its type (_forward_op)."""
    attrs = dict(ref.attrs if attrs is None else attrs)
    op = ref.op
    if op == "nn.conv2d":
        return _op.conv2d(args[0], args[1], strides=attrs["strides"], padding=attrs["padding"],
                          dilation=attrs["dilation"], groups=attrs["groups"], out_dtype=attrs.get("out_dtype", ""))
    if op == "nn.dense":
        return _op.dense(args[0], args[1], out_dtype=attrs.get("out_dtype", ""))
    if op in ("add", "multiply", "right_shift", "left_shift"):
        return getattr(_op, op)(args[0], args[1])
    if op == "cast":
        return Call(op, args, attrs, TensorType(args[0].shape, attrs["dtype"]))
    # shape from the reference call, dtype from the data operand
    return Call(op, args, attrs, TensorType(ref.shape, args[0].dtype))


def _is_constant(e: Expr) -> bool:
    """relay.analysis.check_constant: no free variables."""
    return all(not isinstance(n, Var) for n in post_order(e))


def _sconst(v, dtype) -> Constant:
    return Constant(np.asarray(v, dtype=dtype))


# ----------------------------------------------------------------------------- prerequisites

def prerequisite_optimize(mod, params=None) -> IRModule:
    """quantize.py:312-322: bind params as constants, then SimplifyInference -> FoldConstant ->
    FoldScaleAxis (relay/transform.py: batch norms become a per-channel multiply folded into the
    producing conv / dense weights, plus a constant add) -> CanonicalizeOps (``nn.bias_add`` to
    ``add`` with an expanded bias) -> FoldConstant."""
    from ..transform import fold_scale_axis, simplify_inference
    func = mod["main"] if isinstance(mod, IRModule) else IRModule.from_expr(mod)["main"]
    params = {k: np.asarray(v.numpy() if hasattr(v, "numpy") else v) for k, v in (params or {}).items()}
    bound = {id(v): Constant(params[v.name_hint]) for v in func.params if v.name_hint in params}

    def canon(call: Call, args):
        if call.op == "nn.bias_add":
            x, b = args
            ax = call.attrs["axis"] if call.attrs["axis"] >= 0 else len(x.shape) + call.attrs["axis"]
            shape = (x.shape[ax],) + (1,) * (len(x.shape) - ax - 1)
            b = Constant(b.data.reshape(shape)) if isinstance(b, Constant) else _op.reshape(b, shape)
            return _op.add(x, b)
        if all(x is y for x, y in zip(args, call.args)):
            return call
        return _forward(call, args)

    def bind(call: Call, args):
        args = [bound.get(id(a), a) for a in args]
        if all(x is y for x, y in zip(args, call.args)):
            return call
        return Call(call.op, args, call.attrs, call.checked_type)

    body = rebuild(func.body, bind)
    body = bound.get(id(body), body)
    m = IRModule(Function(_params_of(body, func.params), body))
    m = fold_scale_axis(fold_constant(simplify_inference(m)))
    func = m["main"]
    body = rebuild(func.body, canon)
    return fold_constant(IRModule(Function(_params_of(body, func.params), body)))


# ----------------------------------------------------------------------------- partition

class _QPartition(_Temp):
    def __init__(self, expr: Expr):
        self.expr = expr

    def realize(self) -> Expr:
        # partition.cc:40-46: cast hint + stop fusion
        return _op.stop_fusion(_op.cast_hint(self.expr, current_qconfig().dtype_input))


def _pcheck(e):
    return (True, e.expr) if isinstance(e, _QPartition) else (False, e)


def _p_conv2d(ref, args):
    dcond, data = _pcheck(args[0])
    kcond, kernel = _pcheck(args[1])
    assert not kcond
    if dcond:
        data = args[0].realize()
    return _QPartition(_forward(ref, [data, kernel]))


def _p_identity(ref, args):
    cond, e = _pcheck(args[0])
    return _QPartition(_forward(ref, [e])) if cond else None


def _p_add(ref, args):
    lc, lhs = _pcheck(args[0])
    rc, rhs = _pcheck(args[1])
    if lc and rc:  # the first residual join of a ResNet stage
        return _QPartition(_forward(ref, [args[0].realize(), args[1].realize()]))
    if not lc and rc:  # residual join: lhs is an ended region
        return _forward(ref, [lhs, args[1].realize()])
    if lc and not rc:
        if _is_constant(rhs):  # bias / folded batch norm
            return _QPartition(_forward(ref, [lhs, rhs]))
        return _forward(ref, [args[0].realize(), rhs])  # MobileNetV2-style residual
    return None


def _p_multiply(ref, args):
    lc, _ = _pcheck(args[0])
    rc, rhs = _pcheck(args[1])
    if lc:
        return _QPartition(_forward(ref, [args[0].realize(), rhs]))
    if not rc:
        return None
    raise ValueError("quantize partition: multiply with a quantized rhs")


def _p_gap(ref, args):
    cond, _ = _pcheck(args[0])
    e = args[0].realize() if cond else _QPartition(args[0]).realize()
    return _forward(ref, [e])


_PARTITION_RULES = {"nn.conv2d": _p_conv2d, "clip": _p_identity, "nn.relu": _p_identity,
                    "nn.max_pool2d": _p_identity, "add": _p_add, "multiply": _p_multiply,
                    "nn.global_avg_pool2d": _p_gap}


def partition(mod) -> IRModule:
    func = mod["main"] if isinstance(mod, IRModule) else mod
    return IRModule(_forward_rewrite(func, _PARTITION_RULES))


# ----------------------------------------------------------------------------- annotate

class _QAnnotate(_Temp):
    def __init__(self, expr: Expr, kind: int):
        self.expr, self.kind = expr, kind

    def realize(self) -> Expr:
        return self.expr  # annotate.cc:63


def _akind(e):
    return (e.expr, e.kind) if isinstance(e, _QAnnotate) else (e, None)


class _QuantizeContext:
    """quantize.py:219-262: conv2d counter for ``skip_conv_layers`` and the stop flag."""

    def __init__(self):
        self.qnode_map: Dict[tuple, Call] = {}
        self.conv2d_counter = 0
        self.stopped = False

    def check_to_skip(self, ref: Call) -> bool:
        if self.stopped:
            return True
        skip = current_qconfig().skip_conv_layers
        if skip is not None:
            if self.conv2d_counter in skip and ref.op == "nn.conv2d":
                self.conv2d_counter += 1
                return True
            if ref.op == "nn.conv2d":
                self.conv2d_counter += 1
        return False


def simulated_quantize(data: Expr, dom_scale: Expr, clip_min: Expr, clip_max: Expr, kind: int, sign: bool = True,
                       rounding: str = "round") -> Call:
    return Call(SQ, [data, dom_scale, clip_min, clip_max], {"kind": int(kind), "sign": bool(sign),
                                                            "rounding": rounding}, data.checked_type)


def _attach_sq(ctx: _QuantizeContext, data: Expr, kind: int, sign=True, rounding="round") -> Call:
    """_annotate.py:115-146."""
    if isinstance(data, Call) and data.op == SQ and data.attrs["kind"] == kind and \
            data.attrs["sign"] == sign and data.attrs["rounding"] == rounding:
        return data
    key = (id(data), kind, sign, rounding)
    if key in ctx.qnode_map:
        return ctx.qnode_map[key][1]
    qnode = simulated_quantize(data, Var("dom_scale", ()), Var("clip_min", ()), Var("clip_max", ()), kind, sign,
                               rounding)
    ctx.qnode_map[key] = (data, qnode)  # keeps ``data`` alive so its id stays unique
    return qnode


def _annotate_rules(ctx: _QuantizeContext):
    K = QAnnotateKind

    def guarded(op_name, fn):
        def rule(ref, args):
            if not current_qconfig().guard(ref.op):
                return _forward(ref, [_akind(a)[0] for a in args])
            return fn(ref, args)
        return rule

    def contraction(ref, args):
        if ref.op == "nn.dense" and current_qconfig().skip_dense_layer:
            return None
        if ctx.check_to_skip(ref):
            return None
        lhs, lk = _akind(args[0])
        rhs, rk = _akind(args[1])
        if lk is None or lk == K.ACTIVATION:
            lhs = _attach_sq(ctx, lhs, K.INPUT)
        assert rk is None
        rhs = _attach_sq(ctx, rhs, K.WEIGHT)
        return _QAnnotate(_forward(ref, [lhs, rhs]), K.ACTIVATION)

    def multiply(ref, args):
        if ctx.check_to_skip(ref):
            return None
        lhs, lk = _akind(args[0])
        rhs, rk = _akind(args[1])
        if lk is None and rk is None:
            return None
        if lk in (K.ACTIVATION, K.INPUT) and rk is None:
            if lk == K.ACTIVATION:
                lhs = _attach_sq(ctx, lhs, K.INPUT)
            rhs = _attach_sq(ctx, rhs, K.WEIGHT if _is_constant(rhs) else K.INPUT)
            return _QAnnotate(_forward(ref, [lhs, rhs]), K.ACTIVATION)
        raise ValueError("quantize annotate: unsupported multiply operands")

    def add(ref, args):
        if ctx.check_to_skip(ref):
            return None
        lhs, lk = _akind(args[0])
        rhs, rk = _akind(args[1])
        if lk is None and rk is None:
            return None
        if lk is None:
            assert rk in (K.INPUT, K.ACTIVATION)
            lhs = _attach_sq(ctx, lhs, K.INPUT)
            return _QAnnotate(_forward(ref, [lhs, rhs]), K.INPUT)
        if rk is None:
            rhs = _attach_sq(ctx, rhs, K.WEIGHT if _is_constant(rhs) else K.INPUT)
            return _QAnnotate(_forward(ref, [lhs, rhs]), K.ACTIVATION)
        if lk == K.INPUT and rk == K.INPUT:
            return _QAnnotate(_forward(ref, [lhs, rhs]), K.INPUT)
        if lk == K.ACTIVATION and rk == K.ACTIVATION:
            rhs = _attach_sq(ctx, rhs, K.INPUT)
            return _QAnnotate(_forward(ref, [lhs, rhs]), K.ACTIVATION)
        return _QAnnotate(_forward(ref, [lhs, rhs]), K.ACTIVATION)

    def identity(ref, args):
        if ctx.check_to_skip(ref):
            return None
        x, k = _akind(args[0])
        if k is None:
            return None
        return _QAnnotate(_forward(ref, [x]), k)

    def pool(ref, args):
        if ctx.check_to_skip(ref):
            return None
        x, k = _akind(args[0])
        if k is None:
            return None
        if k == K.ACTIVATION:
            x = _attach_sq(ctx, x, K.INPUT)
        return _QAnnotate(_forward(ref, [x]), K.INPUT)

    def cast_hint(ref, args):
        x, k = _akind(args[0])
        if ctx.check_to_skip(ref):
            return x
        if k is None:
            return args[0]
        if k == K.ACTIVATION:
            x = _attach_sq(ctx, x, K.INPUT)
        return _QAnnotate(_forward(ref, [x]), K.INPUT)

    def gap(ref, args):
        if ctx.check_to_skip(ref):
            return None
        _, k = _akind(args[0])
        if k is None:
            return None
        e = _forward(ref, [_real(args[0])])
        ctx.stopped = True  # quantization stops after global_avg_pool2d (_annotate.py:395-410)
        return e

    rules = {"nn.conv2d": contraction, "nn.dense": contraction, "multiply": multiply, "add": add,
             "nn.max_pool2d": pool, "annotation.cast_hint": cast_hint, "nn.global_avg_pool2d": gap}
    for name in ("reshape", "clip", "nn.relu", "strided_slice", "nn.avg_pool2d", "nn.batch_flatten", "transpose",
                 "annotation.stop_fusion"):
        rules[name] = identity
    return {k: guarded(k, v) for k, v in rules.items()}


def annotate(mod, ctx: Optional[_QuantizeContext] = None) -> IRModule:
    func = mod["main"] if isinstance(mod, IRModule) else mod
    ctx = ctx or _QuantizeContext()

    def multi_ref(e):  # annotate.cc:68-77
        if isinstance(e, _QAnnotate):
            return _QAnnotate(_attach_sq(ctx, e.expr, QAnnotateKind.INPUT), QAnnotateKind.INPUT)
        return e

    return IRModule(_forward_rewrite(func, _annotate_rules(ctx), multi_ref))


# ----------------------------------------------------------------------------- calibrate

def _power2_scale(w: np.ndarray) -> float:
    val = float(np.amax(np.abs(w)))
    return 2 ** math.ceil(math.log(val, 2)) if val > 0 else 1.0


def _max_scale(w: np.ndarray) -> float:
    return float(np.amax(np.abs(w)))


def stats_profile(mod):
    """CreateStatsCollector (src/relay/quantize/calibrate.cc:148-190): every simulated_quantize
    becomes the identity of its input; the inputs of the non-weight ones, in post-order, are the
    values to profile.  Returns (profile module, the profiled expressions)."""
    func = mod["main"] if isinstance(mod, IRModule) else mod
    targets: List[Expr] = []

    def strip(call: Call, args):
        if call.op == SQ:
            if call.attrs["kind"] != QAnnotateKind.WEIGHT:
                assert not isinstance(args[0], Constant)
                targets.append(args[0])
            return args[0]
        return call if all(x is y for x, y in zip(args, call.args)) else _forward(call, args)

    body = rebuild(func.body, strip)
    return IRModule(Function(_params_of(body, func.params), body)), targets


def collect_stats(mod, dataset, chunk_by: int = -1):
    """_calibrate.py:collect_stats: run the profile graph over the dataset on the MI355X (the
    engine records every op output, so each profiled value is read back by its record name) and
    yield, per chunk of layers, the concatenated flattened values."""
    from ..build_module import build
    from ...contrib.graph_executor import GraphModule
    prof, targets = stats_profile(mod)
    body = prof["main"].body
    names: Dict[int, str] = {}
    counter = 0
    for n in post_order(body):
        if isinstance(n, Var):
            names[id(n)] = n.name_hint
        elif isinstance(n, Call):
            names[id(n)] = f"%{counter}"
            counter += 1
    gm = GraphModule(build(prof, target="mi355x")["default"]())
    tnames = [names[id(t)] for t in targets]
    chunk = len(tnames) if chunk_by == -1 else chunk_by
    for i in range(0, len(tnames), chunk):
        outs: List[List[np.ndarray]] = [[] for _ in tnames[i:i + chunk]]
        for batch in dataset:
            gm.set_input(**batch)
            gm.run()
            for j, name in enumerate(tnames[i:i + chunk]):
                outs[j].append(np.asarray(gm.get_node_output(name).numpy()))
        yield [np.concatenate(o).reshape(-1) for o in outs]


def find_scale_by_percentile(arr: np.ndarray, percentile: float = 0.99999) -> float:
    """_calibrate.py:_find_scale_by_percentile."""
    x = np.abs(arr)
    max_k = int(x.size * percentile)
    return float(np.partition(x, max_k)[max_k])


def find_scale_by_kl(arr: np.ndarray, quantized_dtype: str = "int8", num_bins: int = 8001,
                     num_quantized_bins: int = 255, edges_as: str = "reference") -> float:
    """kl_divergence.py:_find_scale_by_kl: a symmetric histogram of the values, then the native
    MinimizeKL (tk_find_scale_by_kl, csrc/tk_calibrate.cc).

    The reference hands np.histogram's edge array to MinimizeKL through a ``c_float*`` cast of its
    buffer (kl_divergence.py:46-51), whatever numpy built: for float32 statistics (every profile
    graph output of a float32 model) those are float32 edges and the cast is exact; for float64
    statistics the C side reads the first num_bins + 1 float32 words of the float64 buffer.
    ``edges_as="reference"`` (default) passes exactly those bytes, so the threshold equals the
    reference's for any input dtype; ``edges_as="values"`` converts the edge values to float32
    instead (a meaningful threshold for float64 statistics, where the reference's is not)."""
    if edges_as not in ("reference", "values"):
        raise ValueError(f"find_scale_by_kl: edges_as must be 'reference' or 'values', not {edges_as!r}")
    import ctypes
    from ... import _lib
    arr = np.asarray(arr)
    min_val, max_val = np.min(arr), np.max(arr)
    thres = max(abs(min_val), abs(max_val))
    if min_val >= 0 and quantized_dtype in ["uint8"]:
        num_quantized_bins = num_quantized_bins * 2 + 1
    hist, edges = np.histogram(arr, bins=num_bins, range=(-thres, thres))
    hist = np.ascontiguousarray(hist, np.int32)
    edges = kl_edge_buffer(edges, num_bins) if edges_as == "reference" else np.ascontiguousarray(edges, np.float32)
    out = ctypes.c_float()
    _lib.check(_lib.load().tk_find_scale_by_kl(hist.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                               edges.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                               num_bins, num_quantized_bins, ctypes.byref(out)),
               "tk_find_scale_by_kl")
    return float(out.value)


def kl_edge_buffer(edges: np.ndarray, num_bins: int) -> np.ndarray:
    """The num_bins + 1 float32 words MinimizeKL reads from np.histogram's edge array after the
    reference's ``ctypes.cast(edges.ctypes.data_as(POINTER(c_float)), c_void_p)``
    (kl_divergence.py:42-48; calibrate.cc:214-218 copies ``hist_edges_ptr[0 .. num_bins]``): the
    array's own bytes reinterpreted, not its values converted."""
    raw = np.ascontiguousarray(edges).view(np.uint8)
    return np.frombuffer(raw.tobytes()[:4 * (num_bins + 1)], np.float32).copy()


def _dataset_scales(mod, dataset, finder) -> List[float]:
    if dataset is None:
        raise ValueError("calibrate: this calibrate_mode needs a dataset (list of {input name: array})")
    cfg = current_qconfig()
    scales: List[float] = []
    for samples in collect_stats(mod, list(dataset), cfg.calibrate_chunk_by):
        scales += [finder(s) for s in samples]
    return scales


def calibrate(mod, dataset=None) -> IRModule:
    """_calibrate.py:158-238 (``_set_params``): per simulated_quantize,
    dom_scale = scale / 2^(nbit - sign), clip = +-(2^(nbit - sign) - 1), all float32; the scale
    is ``global_scale``, or found on the dataset (``kl_divergence``, ``percentile``) for inputs and
    activations, and ``power2`` / ``max`` of the constant for weights."""
    cfg = current_qconfig()
    wfunc = {"power2": _power2_scale, "max": _max_scale}.get(cfg.weight_scale)
    if wfunc is None:
        raise ValueError(f"Unknown weight scale mode {cfg.weight_scale}")
    if cfg.calibrate_mode == "global_scale":
        dataset_scales = None
    elif cfg.calibrate_mode in ("kl_divergence", "percentile"):
        finder = find_scale_by_kl if cfg.calibrate_mode == "kl_divergence" else find_scale_by_percentile
        found = _dataset_scales(mod, dataset, finder)
        n_act = len(stats_profile(mod)[1])
        if len(found) != n_act:
            raise RuntimeError(f"calibrate: {len(found)} profiled scales for {n_act} activation quantizers")
        dataset_scales = iter(found)
    else:
        raise ValueError(f"Unknown calibrate mode {cfg.calibrate_mode}")
    func = mod["main"] if isinstance(mod, IRModule) else mod

    def bind(call: Call, args):
        if call.op != SQ:
            return call if all(x is y for x, y in zip(args, call.args)) else _forward(call, args)
        kind = call.attrs["kind"]
        valid_range = 2 ** (cfg.get_nbit_by_kind(kind) - int(call.attrs["sign"]))
        if kind == QAnnotateKind.WEIGHT:
            if not isinstance(args[0], Constant):
                raise ValueError("calibrate: weight simulated_quantize over a non-constant")
            scale = wfunc(args[0].data)
        else:
            scale = cfg.global_scale if dataset_scales is None else next(dataset_scales)
        consts = [_sconst(scale / valid_range, f32), _sconst(-(valid_range - 1), f32), _sconst(valid_range - 1, f32)]
        return Call(SQ, [args[0]] + consts, call.attrs, call.checked_type)

    body = rebuild(func.body, bind)
    return IRModule(Function(_params_of(body, func.params), body))


# ----------------------------------------------------------------------------- realize

class _QRealizeInt(_Temp):
    def __init__(self, data: Expr, dom_scale, dtype: str):
        self.data, self.dom_scale, self.dtype = data, f32(dom_scale), str(dtype)

    def realize(self) -> Expr:  # realize.cc:45-51: dequantize
        return _op.multiply(_op.cast(self.data, "float32"), _sconst(self.dom_scale, f32))


def _scalar(e: Expr) -> float:
    assert isinstance(e, Constant) and e.data.size == 1, "expected a scalar constant"
    return e.data.reshape(()).item()


def _fixed_point_multiplier_shift(x: float):
    """GetFixedPointMultiplierShift (src/relay/qnn/utils.cc:33-57), the library's host port."""
    import ctypes
    from ... import _lib
    m, sh = ctypes.c_int32(), ctypes.c_int32()
    _lib.check(_lib.load().tk_fixed_point_multiplier_shift(float(x), ctypes.byref(m), ctypes.byref(sh)),
               "tk_fixed_point_multiplier_shift")
    return int(m.value), int(sh.value)


def _mul_and_div(data: Expr, s1, s2, dtype: str) -> Expr:
    """realize.cc:65-92: data * s1 / s2 with a shift where possible."""
    cfg = current_qconfig()
    s1, s2 = f32(s1), f32(s2)
    if s1 == s2:
        return data
    factor = f32(s1 / s2)
    shift_factor = f32(np.log2(factor))
    assert shift_factor > 0
    if int(shift_factor) == shift_factor:
        return _op.left_shift(data, _sconst(int(shift_factor), dtype))
    if int(factor) == factor:
        return _op.multiply(data, _sconst(factor, dtype))
    if cfg.rounding != "UPWARD":
        raise UnsupportedError("quantize realize: TONEAREST fixed-point multiply")
    m, sh = _fixed_point_multiplier_shift(float(factor))
    return _op.cast(_op.fixed_point_multiply(data, m, sh), dtype)


def _realize_rules():
    cfg = current_qconfig()

    def sq(ref, args):
        assert ref.attrs["rounding"] == "round"
        dom = f32(_scalar(args[1]))
        cmin, cmax = float(f32(_scalar(args[2]))), float(f32(_scalar(args[3])))
        n = args[0]
        if isinstance(n, _QRealizeInt):
            data = n.data
            idom, odom = n.dom_scale, dom
            if idom == odom:
                return _QRealizeInt(_op.clip(data, cmin, cmax), dom, n.dtype)
            shift_nbit = f32(np.log2(f32(odom / idom)))
            assert shift_nbit != 0
            if int(shift_nbit) == shift_nbit:
                if shift_nbit > 0:
                    if cfg.round_for_shift:
                        data = _op.add(data, _sconst(int(2.0 ** (float(shift_nbit) - 1)), cfg.dtype_activation))
                    data = _op.right_shift(data, _sconst(int(shift_nbit), cfg.dtype_activation))
                else:
                    data = _op.left_shift(data, _sconst(int(-shift_nbit), cfg.dtype_activation))
                return _QRealizeInt(_op.clip(data, cmin, cmax), dom, n.dtype)
            if cfg.rounding != "UPWARD":
                raise UnsupportedError("quantize realize: TONEAREST fixed-point multiply")
            data = _op.cast(data, "int64")
            m, sh = _fixed_point_multiplier_shift(float(f32(idom / odom)))
            data = _op.fixed_point_multiply(data, m, sh)
            return _QRealizeInt(_op.cast(_op.clip(data, cmin, cmax), n.dtype), dom, n.dtype)
        assert not isinstance(n, _Temp)
        scaled = _op.multiply(n, _sconst(f32(1) / dom, f32))
        return _QRealizeInt(_op.clip(_op.round(scaled), cmin, cmax), dom, "float32")

    def contraction(ref, args):
        lhs, rhs = args
        if ref.op == "nn.dense" and not (isinstance(lhs, _Temp) and isinstance(rhs, _Temp)):
            return None
        if not (isinstance(lhs, _QRealizeInt) and isinstance(rhs, _QRealizeInt)):
            assert not (isinstance(lhs, _Temp) and isinstance(rhs, _Temp))
            return None
        ldata = lhs.data if lhs.dtype == cfg.dtype_input else _op.cast(lhs.data, cfg.dtype_input)
        rdata = _op.cast(rhs.data, cfg.dtype_weight)
        attrs = dict(ref.attrs, out_dtype=cfg.dtype_activation)
        ret = _forward(ref, [ldata, rdata], attrs)
        return _QRealizeInt(ret, f32(lhs.dom_scale * rhs.dom_scale), cfg.dtype_activation)

    def multiply(ref, args):
        lhs, rhs = args
        if isinstance(lhs, _QRealizeInt) and isinstance(rhs, _QRealizeInt):
            dt = cfg.dtype_activation
            ld = lhs.data if lhs.dtype == dt else _op.cast(lhs.data, dt)
            rd = rhs.data if rhs.dtype == dt else _op.cast(rhs.data, dt)
            return _QRealizeInt(_forward(ref, [ld, rd]), f32(lhs.dom_scale * rhs.dom_scale), dt)
        assert not (isinstance(lhs, _Temp) and isinstance(rhs, _Temp))
        return None

    def unify(ref_args, args, dtype):
        """UnifyDTypeScale (realize.cc:300-345) for two operands."""
        ret = []
        for ref_arg, n in zip(ref_args, args):
            d = n.data
            if n.dtype != dtype:
                d = _op.cast(d, dtype)
            elif isinstance(ref_arg, Call) and ref_arg.op == SQ and ref_arg.attrs["kind"] == QAnnotateKind.INPUT:
                d = _op.cast(_op.stop_fusion(_op.cast(d, cfg.dtype_input)), dtype)
            ret.append(d)
        s = min(args[0].dom_scale, args[1].dom_scale)  # ChooseDomScale
        ret = [_mul_and_div(d, n.dom_scale, s, dtype) for d, n in zip(ret, args)]
        return ret, f32(s)

    def add(ref, args):
        lhs, rhs = args
        if isinstance(lhs, _QRealizeInt) and isinstance(rhs, _QRealizeInt):
            ret, s = unify(ref.args, args, cfg.dtype_activation)
            ret = [_op.stop_fusion(d) if n.dtype == "float32" else d for d, n in zip(ret, args)]
            return _QRealizeInt(_forward(ref, ret), s, cfg.dtype_activation)
        if isinstance(lhs, _Temp) or isinstance(rhs, _Temp):
            raise ValueError("quantize realize: add of a quantized and an unquantized operand")
        return None

    def clip(ref, args):
        n = args[0]
        if isinstance(n, _QRealizeInt):
            dom = float(n.dom_scale)
            attrs = {"a_min": ref.attrs["a_min"] / dom, "a_max": ref.attrs["a_max"] / dom}
            return _QRealizeInt(_forward(ref, [n.data], attrs), n.dom_scale, n.dtype)
        return None

    def identity(ref, args):
        n = args[0]
        if isinstance(n, _QRealizeInt):
            return _QRealizeInt(_forward(ref, [n.data]), n.dom_scale, n.dtype)
        return None

    def cast_input(ref, args):  # max pool: realize.cc:441-451
        n = args[0]
        if isinstance(n, _QRealizeInt):
            return _QRealizeInt(_forward(ref, [_op.cast(n.data, cfg.dtype_input)]), n.dom_scale, cfg.dtype_input)
        return None

    def avg_pool(ref, args):
        n = args[0]
        if isinstance(n, _QRealizeInt):
            d = n.data if n.dtype == cfg.dtype_activation else _op.cast(n.data, cfg.dtype_activation)
            return _QRealizeInt(_forward(ref, [d]), n.dom_scale, cfg.dtype_activation)
        return None

    def cast_hint(ref, args):
        n = args[0]
        if isinstance(n, _QRealizeInt):
            dt = ref.attrs["dtype"]
            return _QRealizeInt(_op.cast(n.data, dt), n.dom_scale, dt)
        return None

    rules = {SQ: sq, "nn.conv2d": contraction, "nn.dense": contraction, "multiply": multiply, "add": add,
             "clip": clip, "nn.max_pool2d": cast_input, "nn.avg_pool2d": avg_pool,
             "nn.global_avg_pool2d": avg_pool, "annotation.cast_hint": cast_hint}
    for name in ("nn.relu", "reshape", "strided_slice", "nn.batch_flatten", "transpose", "annotation.stop_fusion"):
        rules[name] = identity
    return rules


def realize(mod) -> IRModule:
    func = mod["main"] if isinstance(mod, IRModule) else mod
    return IRModule(_forward_rewrite(func, _realize_rules()))


# ----------------------------------------------------------------------------- driver

def quantize(mod, params=None, dataset=None) -> IRModule:
    """quantize.py:330-379: prerequisite_optimize -> partition -> annotate -> calibrate ->
    [realize] -> FoldConstant, under the current ``qconfig``."""
    cfg = current_qconfig()
    if cfg.partition_conversions not in ("disabled", "enabled", "fully_integral"):
        raise ValueError(f"partition_conversions={cfg.partition_conversions!r}")
    mod = prerequisite_optimize(mod, params)
    mod = partition(mod)
    mod = annotate(mod, _QuantizeContext())
    mod = calibrate(mod, dataset)
    if not cfg.do_simulation:
        mod = realize(mod)
    mod = fold_constant(mod)
    if cfg.partition_conversions != "disabled":
        # quantize.py:373-377
        from .partition_conversions import partition_conversions
        qd = {cfg.dtype_input, cfg.dtype_weight, cfg.dtype_activation}
        return partition_conversions(mod, qd, cfg.partition_conversions == "fully_integral")
    return mod

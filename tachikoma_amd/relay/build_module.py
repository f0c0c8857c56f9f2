"""``relay.build`` for the MI355X engine.

Reference surface: ``relay.build(ir_mod, target, params)``
(python/tvm/relay/build_module.py:409-419) → ``lib["default"](dev)`` →
``graph_executor.GraphModule`` (python/tvm/contrib/graph_executor.py:114-351).

Lowering is split in two:
  * ``lower(mod, params)`` → ``Plan``: topologically ordered ops named the way
    MRT names symbols (``%N`` in post-order, python/tvm/mrt/symbol.py:212-253,
    utils.py:29-67), with every QNN constant folded the way the reference's
    canonicalisation folds it.  Pure host code (no GPU needed).
  * ``ExecutorFactory(plan, params)["default"](dev)`` → a device module: one HBM
    buffer per op output (no storage reuse, so every output stays traceable),
    weights uploaded/packed once, and a native ``tk_module`` node list.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .. import _lib
from .expr import Call, Constant, Expr, Function, IRModule, Tuple, Var, post_order
from .op import INT_DTYPES
from .qnn import op as _qnn

TARGETS = ("mi355x", "rocm", "hip", "gfx950")


class UnsupportedError(NotImplementedError):
    pass


@dataclass
class PlanTensor:
    name: str
    shape: Tuple[int, ...]
    dtype: str

    @property
    def nbytes(self) -> int:
        return int(np.prod(self.shape, dtype=np.int64)) * np.dtype(self.dtype).itemsize


@dataclass
class PlanOp:
    index: int
    name: str
    op: str
    inputs: List[str]
    attrs: Dict[str, Any]
    out: PlanTensor
    consts: Dict[str, np.ndarray] = field(default_factory=dict)

    def describe(self) -> Dict[str, Any]:
        def py(v):
            if isinstance(v, np.ndarray):
                return v.tolist()
            if isinstance(v, (np.integer,)):
                return int(v)
            if isinstance(v, (np.floating,)):
                return float(v)
            if isinstance(v, tuple):
                return list(v)
            return v
        d = {"id": self.index, "name": self.name, "op": self.op, "inputs": list(self.inputs),
             "shape": list(self.out.shape), "dtype": self.out.dtype,
             "attrs": {k: py(v) for k, v in self.attrs.items()}}
        if self.consts:
            d["consts"] = {k: py(v) for k, v in self.consts.items()}
        return d


@dataclass
class Plan:
    inputs: List[PlanTensor]
    params: List[PlanTensor]
    ops: List[PlanOp]
    outputs: List[str]

    def tensor(self, name: str) -> PlanTensor:
        for t in self.inputs + self.params:
            if t.name == name:
                return t
        for o in self.ops:
            if o.name == name:
                return o.out
        raise KeyError(name)

    @property
    def records(self) -> List[PlanTensor]:
        """Traced tensors in file order: graph inputs, then every op output (topo order)."""
        return list(self.inputs) + [o.out for o in self.ops]


def _scalar(c: Expr, what: str):
    if not isinstance(c, Constant):
        raise UnsupportedError(f"{what} must be a relay.const")
    return c.data


def _resolve_rounding(attrs) -> Tuple[str, str]:
    """SelectRequntizeParameter (src/relay/qnn/utils.cc:218-229) with the pinned defaults
    (requantize_config.h:53-72: rounding UPWARD, compute_dtype int64 for llvm w/o -mcpu)."""
    r = attrs.get("rounding", "None")
    if r in (None, "None"):
        r = attrs.get("cfg_rounding") or "UPWARD"
    cd = attrs.get("compute_dtype", "None")
    if cd in (None, "None"):
        cd = attrs.get("cfg_compute_dtype") or "int64"
    if r not in ("UPWARD", "TONEAREST"):
        raise ValueError(f"qnn.requantize: rounding must be UPWARD or TONEAREST, got {r}")
    if cd not in ("int64", "float32", "float64"):
        # RequantizeLower's check (requantize.cc:389-392)
        raise ValueError(f"qnn.requantize: compute_dtype must be int64, float32 or float64, got {cd}")
    return r, cd


def fp_requantize_plan(input_scale, output_scale) -> Tuple[int, float, Optional[np.ndarray]]:
    """RequantizeLowerFP's constants (src/relay/qnn/op/requantize.cc:310-341): per-tensor, the
    double multiplier double(s_in) / double(s_out) and whether it is applied at all (skipped when
    the two float32 scales are structurally equal, :313); per-axis, one double per channel (always
    applied).  The kernel converts them to the compute type as MakeConstantScalar /
    MakeConstantTensor do.  Returns (scaled, multiplier, multipliers or None)."""
    s_in = np.asarray(input_scale, dtype=np.float32)
    s_out = np.float32(output_scale)
    if s_in.ndim == 0:
        scaled = int(not _is_equal_scalar(s_in, np.asarray(s_out)))
        return scaled, float(np.float64(s_in)) / float(np.float64(s_out)), None
    ms = np.array([float(np.float64(v)) / float(np.float64(s_out)) for v in s_in.reshape(-1)], dtype=np.float64)
    return 1, 0.0, ms


def _fp_side(a: Dict[str, Any], consts: Dict[str, np.ndarray], side: str, s_in, s_out, axis: int, nd: int,
             cd: str) -> None:
    """The RequantizeLowerFP constants of one inner requantize into attrs ``{side}_fp_*`` and the
    per-axis const ``{side}_fp_multipliers`` (zero points stay in ``{side}_zero_point(s)``)."""
    scaled, m, ms = fp_requantize_plan(s_in, s_out)
    a[f"{side}_fp_bits"] = 32 if cd == "float32" else 64
    a[f"{side}_fp_scaled"] = scaled
    a[f"{side}_fp_multiplier"] = m
    a[f"{side}_axis"] = _norm_axis(axis, nd)
    if ms is not None:
        consts[f"{side}_fp_multipliers"] = ms


def requantize_plan(input_scale: np.ndarray, output_scale, rounding: str):
    """Fold scales into (mode, multipliers, shifts) through the library's host port of
    RequantizeLowerInt's constant folding (tk_requantize_prepare)."""
    lib = _lib.load()
    s_in = np.asarray(input_scale, dtype=np.float32)
    per_axis = s_in.ndim != 0
    vals = s_in.reshape(-1) if per_axis else s_in.reshape(1)
    n = len(vals) if per_axis else 0
    cap = max(1, len(vals))
    ms = (ctypes.c_int32 * cap)()
    ss = (ctypes.c_int32 * cap)()
    mode = ctypes.c_int()
    arr = (ctypes.c_float * len(vals))(*[float(v) for v in vals])
    rnd = _lib.TK_ROUND_UPWARD if rounding == "UPWARD" else _lib.TK_ROUND_TONEAREST
    _lib.check(lib.tk_requantize_prepare(arr, n, ctypes.c_float(float(np.float32(output_scale))), rnd, ms, ss,
                                         ctypes.byref(mode)), "tk_requantize_prepare")
    return int(mode.value), np.array(ms[:cap], dtype=np.int32), np.array(ss[:cap], dtype=np.int32)


def fixed_point_multiplier_shift(v: float) -> Tuple[int, int]:
    """GetFixedPointMultiplierShift (src/relay/qnn/utils.cc:33-57) of a double, through the
    library's host port (tk_fixed_point_multiplier_shift)."""
    m, s = ctypes.c_int32(), ctypes.c_int32()
    _lib.check(_lib.load().tk_fixed_point_multiplier_shift(ctypes.c_double(float(v)), ctypes.byref(m), ctypes.byref(s)),
               "tk_fixed_point_multiplier_shift")
    return int(m.value), int(s.value)


def _clip_bound(v: float, dtype: str) -> int:
    info = np.iinfo(np.dtype(dtype))
    if not np.isfinite(v):
        return int(info.max) if v > 0 else int(info.min)
    iv = int(np.trunc(v))
    return max(min(iv, int(info.max)), int(info.min))


def lower(mod, params: Optional[Dict[str, Any]] = None) -> Plan:
    """Topologically order the graph, name ops MRT-style and fold QNN constants."""
    func = mod["main"] if isinstance(mod, IRModule) else IRModule.from_expr(mod)["main"]
    params = {k: np.asarray(v.numpy() if hasattr(v, "numpy") else v) for k, v in (params or {}).items()}
    nodes = post_order(func.body)
    names: Dict[int, str] = {}
    inputs: List[PlanTensor] = []
    plist: List[PlanTensor] = []
    ops: List[PlanOp] = []
    counter = 0
    for v in func.params:
        if not isinstance(v, Var):
            continue
    for node in nodes:
        if isinstance(node, Var):
            names[id(node)] = node.name_hint
            t = PlanTensor(node.name_hint, node.shape, node.dtype)
            if node.name_hint in params:
                p = params[node.name_hint]
                if tuple(p.shape) != node.shape:
                    raise TypeError(f"param {node.name_hint}: shape {p.shape} vs {node.shape}")
                plist.append(t)
            else:
                inputs.append(t)
        elif isinstance(node, (Constant, Tuple)):
            continue  # a tuple is no op: no record, no symbol name (expr.Tuple)
        elif _folded_const(node) is not None:
            # reshape of a constant (the simulated_(de)quantize constructors' [-1] reshapes): the
            # reference's FoldConstant makes it a constant when the graph is built -- no op, no name
            names[id(node)] = None
        elif isinstance(node, Call):
            name = f"%{counter}"
            counter += 1
            names[id(node)] = name
            ops.append(_lower_call(len(ops), name, node, names))
        else:
            raise UnsupportedError(f"expression type {type(node).__name__}")
    # free vars not reachable from the body are ignored like Relay does for unused params
    out = names[id(func.body)]
    return Plan(inputs, plist, ops, [out])


def _folded_const(e: Expr) -> Optional[np.ndarray]:
    """The value of a constant or of ``reshape(constant)`` (which FoldConstant folds), else None."""
    if isinstance(e, Constant):
        return e.data
    if isinstance(e, Call) and e.op == "reshape" and isinstance(e.args[0], Constant):
        return np.reshape(e.args[0].data, e.shape)
    return None


def _tensor_args(call: Call, k: int, names) -> List[str]:
    out = []
    for a in call.args[:k]:
        if isinstance(a, Constant) or names.get(id(a), "") is None:
            raise UnsupportedError(f"{call.op}: constant tensor operands must be passed as params (MRT symbols)")
        out.append(names[id(a)])
    return out


def _is_equal_scalar(x: np.ndarray, y: np.ndarray) -> bool:
    """IsEqualScalar (src/relay/qnn/utils.h): both rank-0, same dtype, same bytes."""
    x, y = np.asarray(x), np.asarray(y)
    return x.ndim == 0 and y.ndim == 0 and x.dtype == y.dtype and x.tobytes() == y.tobytes()


def _norm_axis(axis: int, nd: int) -> int:
    return axis + nd if axis < 0 else axis if nd else 0


def _rq_side(a: Dict[str, Any], consts: Dict[str, np.ndarray], side: str, s_in, zp_in, s_out, zp_out, axis: int,
             nd: int, rounding: str) -> None:
    """One requantize plan (RequantizeLowerInt constants: mode, multiplier(s), shift(s), zero
    point(s)) into attrs ``{side}_*`` and per-axis consts ``{side}_multipliers`` / ``_shifts`` /
    ``_zero_points``.  ``axis`` indexes the operand (rank ``nd``)."""
    s_in = np.asarray(s_in, np.float32)
    zp_in = np.asarray(zp_in, np.int32)
    mode, ms, ss = requantize_plan(s_in if s_in.ndim else np.float32(s_in), np.float32(s_out), rounding)
    a[f"{side}_mode"] = mode
    a[f"{side}_axis"] = _norm_axis(axis, nd)
    if mode >= _lib.TK_RQ_AXIS_UPWARD:
        consts[f"{side}_multipliers"], consts[f"{side}_shifts"] = ms, ss
        a[f"{side}_multiplier"] = a[f"{side}_shift"] = 0
    else:
        a[f"{side}_multiplier"], a[f"{side}_shift"] = int(ms[0]), int(ss[0])
    if zp_in.ndim == 0:
        a[f"{side}_zero_point"] = int(zp_in)
    else:
        a[f"{side}_zero_point"] = 0
        consts[f"{side}_zero_points"] = zp_in.reshape(-1).astype(np.int32)
    a["output_zero_point"] = int(np.asarray(zp_out))


def _qnn_rounding(a: Dict[str, Any], float_ok: bool = False) -> str:
    """The requantize rounding a QNN canonicalization's inner ``Requantize`` gets: the
    requantize_config in effect when the op was built, else UPWARD (qnn/utils.h:106-122).  The
    config's compute_dtype goes to ``a["compute_dtype"]``; a float one is implemented for
    qnn.add / subtract / mul (``float_ok``) and refused elsewhere."""
    r = a.pop("cfg_rounding", None) or "UPWARD"
    cd = a.pop("cfg_compute_dtype", None) or "int64"
    if cd not in ("int64", "float32", "float64"):
        raise ValueError(f"compute_dtype must be int64, float32 or float64, got {cd}")
    if cd != "int64" and not float_ok:
        raise UnsupportedError(f"compute_dtype={cd}: the float requantize form is implemented for qnn.requantize, "
                               "qnn.add, qnn.subtract and qnn.mul only")
    a["compute_dtype"] = cd
    return r


def _lower_binary(call: Call, a: Dict[str, Any], consts: Dict[str, np.ndarray]) -> None:
    """qnn.add / qnn.subtract (RequantizeOrUpcast of both sides, op_common.h:193-207) and qnn.mul
    (mul.cc:43-159) into requantize plans for the device's tk_qnn_binary."""
    op = call.op
    lhs, rhs = call.args[0], call.args[1]
    vals = [_scalar(call.args[i], f"{op} param") for i in range(2, 8)]
    ls, lz, rs, rz, os_, oz = [np.asarray(v) for v in vals]
    rounding = _qnn_rounding(a, float_ok=True)
    a["rounding"] = rounding
    cd = a["compute_dtype"]
    ln, rn = len(lhs.shape), len(rhs.shape)
    if op in ("qnn.add", "qnn.subtract"):
        for side, s_, z_, ax, nd in (("lhs", ls, lz, a["lhs_axis"], ln), ("rhs", rs, rz, a["rhs_axis"], rn)):
            up = _is_equal_scalar(s_.astype(np.float32), os_.astype(np.float32)) and \
                _is_equal_scalar(z_.astype(np.int32), oz.astype(np.int32))
            a[f"{side}_upcast"] = int(up)
            if up:
                a.update({f"{side}_mode": 0, f"{side}_multiplier": 0, f"{side}_shift": 0,
                          f"{side}_zero_point": int(z_), f"{side}_axis": 0})
            else:
                _rq_side(a, consts, side, s_, z_, os_, oz, ax, nd, rounding)
                if cd != "int64":
                    _fp_side(a, consts, side, s_, os_, ax, nd, cd)
        a["output_zero_point"] = int(oz)
        # scalar floats for the fused residual-join kernels (add_block / conv-block join)
        a.update(lhs_scale=float(np.float32(ls)) if ls.ndim == 0 else None,
                 rhs_scale=float(np.float32(rs)) if rs.ndim == 0 else None, output_scale=float(np.float32(os_)))
        a["per_tensor"] = int(not consts and lhs.shape == rhs.shape == call.shape)
        return
    # qnn.mul
    a["lhs_upcast"] = a["rhs_upcast"] = 0
    if ls.ndim == 0 and rs.ndim == 0:
        # per-tensor: Requantize(Q', s_a * s_b (a float32 product), 0 -> s_out, zp_out); vector zero
        # points are subtracted as written, i.e. broadcast along the operand's last axis
        for side, z_, x in (("lhs", lz, lhs), ("rhs", rz, rhs)):
            if z_.ndim and (not x.shape or z_.reshape(-1).shape[0] != x.shape[-1]):
                raise UnsupportedError(f"qnn.mul: a {side} zero point of shape {z_.shape} for {x.shape}")
        new_scale = np.float32(np.float32(ls) * np.float32(rs))
        out_axis = -1
    else:
        if a["lhs_axis"] != a["rhs_axis"]:
            raise UnsupportedError("qnn.mul: lhs_axis and rhs_axis differ (mul.cc:154-156)")
        if ls.ndim == 0 or rs.ndim == 0 or ls.size != rs.size:
            raise UnsupportedError("qnn.mul: per-channel scales on both sides, of equal length")
        new_scale = np.array([float(np.float64(x) * np.float64(y)) for x, y in
                              zip(ls.reshape(-1), rs.reshape(-1))], dtype=np.float32)
        out_axis = a["lhs_axis"]
    for side, z_, ax, nd in (("lhs", lz, a["lhs_axis"] if ls.ndim else -1, ln),
                             ("rhs", rz, a["rhs_axis"] if ls.ndim else -1, rn)):
        a[f"{side}_axis"] = _norm_axis(ax, nd)
        a[f"{side}_mode"], a[f"{side}_multiplier"], a[f"{side}_shift"] = 0, 0, 0
        if z_.ndim == 0:
            a[f"{side}_zero_point"] = int(z_)
        else:
            a[f"{side}_zero_point"] = 0
            consts[f"{side}_zero_points"] = z_.reshape(-1).astype(np.int32)
    _rq_side(a, consts, "out", new_scale, np.int32(0), os_, oz, out_axis, ln, rounding)
    if cd != "int64":
        _fp_side(a, consts, "out", new_scale, os_, out_axis, ln, cd)
    a["per_tensor"] = 0


def _lower_call(index: int, name: str, call: Call, names) -> PlanOp:
    op = call.op
    out = PlanTensor(name, call.shape, call.dtype)
    a = dict(call.attrs)
    consts: Dict[str, np.ndarray] = {}
    if op == "qnn.conv2d":
        ins = _tensor_args(call, 2, names)
        za = _scalar(call.args[2], "qnn.conv2d input_zero_point")
        zw = _scalar(call.args[3], "qnn.conv2d kernel_zero_point")
        if np.ndim(za) != 0:
            raise UnsupportedError("qnn.conv2d: per-channel input zero point")
        a["input_zero_point"] = int(za)
        if np.ndim(zw) == 0:
            a["kernel_zero_point"] = int(zw)
        else:
            a["kernel_zero_point"] = 0
            # one per O-dim entry of the kernel; a depthwise-multiplier kernel (C, M, KH, KW) has C
            # of them, each shared by the M output channels c * M + m
            consts["kernel_zero_points"] = np.repeat(np.asarray(zw, np.int32).reshape(-1),
                                                     a.get("depthwise_multiplier", 1))
        a["input_scale"] = _scalar(call.args[4], "scale").tolist()
        a["kernel_scale"] = _scalar(call.args[5], "scale").tolist()
    elif op == "qnn.dense":
        ins = _tensor_args(call, 2, names)
        za = _scalar(call.args[2], "qnn.dense input_zero_point")
        zw = _scalar(call.args[3], "qnn.dense kernel_zero_point")
        if np.ndim(za) != 0:
            raise UnsupportedError("qnn.dense: per-channel input zero point")
        a["input_zero_point"] = int(za)
        if np.ndim(zw) == 0:
            a["kernel_zero_point"] = int(zw)
        else:
            a["kernel_zero_point"] = 0
            consts["kernel_zero_points"] = np.asarray(zw, np.int32).reshape(-1)
        a["input_scale"] = _scalar(call.args[4], "scale").tolist()
        a["kernel_scale"] = _scalar(call.args[5], "scale").tolist()
    elif op == "qnn.requantize":
        ins = _tensor_args(call, 1, names)
        s_in = _scalar(call.args[1], "qnn.requantize input_scale")
        zp_in = _scalar(call.args[2], "qnn.requantize input_zero_point")
        s_out = _scalar(call.args[3], "qnn.requantize output_scale")
        zp_out = _scalar(call.args[4], "qnn.requantize output_zero_point")
        if np.ndim(zp_out) != 0:
            raise UnsupportedError("qnn.requantize: per-axis output zero point")
        rounding, cd = _resolve_rounding(a)
        mode, ms, ss = requantize_plan(s_in, s_out, rounding)
        nd = len(call.args[0].shape)
        axis = a["axis"]
        ax = axis if axis >= 0 else (nd + axis if nd > 0 else 0)
        a.update(rounding=rounding, compute_dtype=cd, mode=mode, channel_axis=ax,
                 input_scale=np.asarray(s_in, np.float32).tolist(), output_scale=float(np.float32(s_out)),
                 output_zero_point=int(zp_out))
        for k in ("cfg_rounding", "cfg_compute_dtype"):
            a.pop(k, None)
        if mode >= _lib.TK_RQ_AXIS_UPWARD:
            consts["multipliers"] = ms
            consts["shifts"] = ss
        else:
            a["multiplier"] = int(ms[0])
            a["shift"] = int(ss[0])
        if cd != "int64":
            # RequantizeLowerFP<32|64> (requantize.cc:293-373): the device runs tk_requantize_fp
            scaled, m, fms = fp_requantize_plan(s_in, s_out)
            a.update(fp_bits=32 if cd == "float32" else 64, fp_scaled=scaled, fp_multiplier=m)
            if fms is not None:
                consts["fp_multipliers"] = fms
        if np.ndim(zp_in) == 0:
            a["input_zero_point"] = int(zp_in)
        else:
            a["input_zero_point"] = 0
            consts["input_zero_points"] = np.asarray(zp_in, np.int32).reshape(-1)
    elif op in ("qnn.add", "qnn.subtract", "qnn.mul"):
        ins = _tensor_args(call, 2, names)
        _lower_binary(call, a, consts)
    elif op == "qnn.concatenate":
        tup = call.args[0]
        if not isinstance(tup, Tuple):
            raise UnsupportedError("qnn.concatenate: the data must be a tuple expression")
        if any(isinstance(f, Constant) for f in tup.fields):
            raise UnsupportedError("qnn.concatenate: constant tensor operands must be passed as params (MRT symbols)")
        ins = [names[id(f)] for f in tup.fields]
        if len(ins) > _lib.CONCAT_MAX:
            raise UnsupportedError(f"qnn.concatenate: at most {_lib.CONCAT_MAX} inputs")
        rounding = _qnn_rounding(a)
        s_out = np.asarray(_scalar(call.args[3], "qnn.concatenate output_scale"), np.float32)
        z_out = np.asarray(_scalar(call.args[4], "qnn.concatenate output_zero_point"), np.int32)
        plans = []
        for sc, zc in zip(call.args[1].fields, call.args[2].fields):
            s_i = np.asarray(_scalar(sc, "qnn.concatenate input scale"), np.float32)
            z_i = np.asarray(_scalar(zc, "qnn.concatenate input zero point"), np.int32)
            same = _is_equal_scalar(s_i, s_out) and _is_equal_scalar(z_i, z_out)
            mode, ms, ss = requantize_plan(s_i, s_out, rounding)
            plans.append({"requant": int(not same), "mode": mode, "multiplier": int(ms[0]), "shift": int(ss[0]),
                          "input_zero_point": int(z_i), "output_zero_point": int(z_out)})
        a.update(axis=_norm_axis(a["axis"], len(call.shape)), rounding=rounding, inputs=plans)
    elif op in ("qnn.quantize", "qnn.dequantize"):
        ins = _tensor_args(call, 1, names)
        sv = np.asarray(_scalar(call.args[1], f"{op} scale"), np.float32)
        zv = np.asarray(_scalar(call.args[2], f"{op} zero point"), np.int32)
        nd = len(call.shape)
        a["axis"] = _norm_axis(a["axis"], nd)
        if sv.size == 1:
            a["scale"] = float(sv.reshape(-1)[0])
        else:
            a["scale"] = 0.0
            consts["scales"] = sv.reshape(-1)
        if zv.size == 1:
            a["zero_point"] = int(zv.reshape(-1)[0])
        else:
            a["zero_point"] = 0
            consts["zero_points"] = zv.reshape(-1)
    elif op in ("qnn.simulated_quantize", "qnn.simulated_dequantize"):
        # topi.nn.simulated_(de)quantize (python/tvm/topi/nn/qnn.py:40-190): the dtype code, scale
        # and zero point are tensors -- constants (folded, uploaded with the node) or graph tensors
        # (read on the device when the node runs, so the dtype may be chosen at run time)
        ins = _tensor_args(call, 1, names)
        if call.args[0].dtype != "float32" or len(call.shape) < 1:
            raise UnsupportedError(f"{op}: float32 data of rank >= 1")
        a["axis"] = _norm_axis(a.get("axis", -1), len(call.shape))
        if not 0 <= a["axis"] < len(call.shape):
            raise TypeError(f"{op}: axis {a['axis']} out of range for {call.shape}")
        srcs = {}
        for k, (key, dt) in enumerate((("dtype_code", np.int32), ("scales", np.float32), ("zero_points", np.int32)),
                                      start=1):
            arg = call.args[k]
            v = _folded_const(arg)
            if arg.dtype != np.dtype(dt).name:
                raise TypeError(f"{op}: {key} must be {np.dtype(dt).name}, got {arg.dtype}")
            if v is not None:
                consts[key] = np.asarray(v, dt).reshape(-1)
                srcs[key] = -1
            else:
                ins.append(names[id(arg)])
                srcs[key] = len(ins) - 1
            n = int(np.prod(arg.shape)) if arg.shape else 1
            if n < 1 or (key == "dtype_code" and n != 1):
                raise TypeError(f"{op}: {key} has {n} values")
            a["n_" + key] = n
        a["sources"] = srcs
    elif op == "qnn.leaky_relu":
        # QnnLeakyReluCanonicalize (leaky_relu.cc:85-140): RequantizeOrUpcast to the output params,
        # then the alpha / (1 - alpha) fixed-point multiplies
        ins = _tensor_args(call, 1, names)
        s_in, z_in, s_out, z_out = (_scalar(call.args[i], "qnn.leaky_relu param") for i in range(1, 5))
        rounding = _qnn_rounding(a)
        up = _is_equal_scalar(s_in, s_out) and _is_equal_scalar(z_in, z_out)
        mode, ms, ss = requantize_plan(np.float32(s_in), np.float32(s_out), rounding)
        a.update(rounding=rounding, upcast=int(up), mode=mode, multiplier=int(ms[0]), shift=int(ss[0]),
                 input_zero_point=int(z_in), output_zero_point=int(z_out), input_scale=float(np.float32(s_in)),
                 output_scale=float(np.float32(s_out)))
        am, as_ = fixed_point_multiplier_shift(a["alpha"])
        zm, zs = fixed_point_multiplier_shift(1.0 - a["alpha"])
        if (am, as_) == (1 << 30, 1) or (zm, zs) == (1 << 30, 1):
            # q_multiply_shift's power-of-two branch needs 1 << -1 there (intrin_rule.cc:231): the
            # reference's compiler rejects the shift amount, so the graph does not build
            raise UnsupportedError(f"qnn.leaky_relu: alpha={a['alpha']} (a fixed_point_multiply by 1.0) does not "
                                   "build in the reference")
        a.update(alpha_multiplier=am, alpha_shift=as_, zp_multiplier=zm, zp_shift=zs)
    elif op in _qnn.UNARY_OPS:
        # legalized to a 256-entry table lookup (legalizations.py:54-86); the device module builds
        # the table (relay/qnn/legalize.py)
        ins = _tensor_args(call, 1, names)
        s_in, z_in, s_out, z_out = (_scalar(call.args[i], f"{op} param") for i in range(1, 5))
        a.update(in_scale=float(np.float32(s_in)), in_zero_point=int(z_in), out_scale=float(np.float32(s_out)),
                 out_zero_point=int(z_out))
    elif op == "qnn.batch_matmul":
        ins = _tensor_args(call, 2, names)
        a.update(input_zero_point=int(_scalar(call.args[2], "qnn.batch_matmul x_zero_point")),
                 kernel_zero_point=int(_scalar(call.args[3], "qnn.batch_matmul y_zero_point")),
                 x_scale=float(np.float32(_scalar(call.args[4], "scale"))),
                 y_scale=float(np.float32(_scalar(call.args[5], "scale"))))
    elif op == "qnn.conv2d_transpose":
        ins = _tensor_args(call, 2, names)
        za = np.asarray(_scalar(call.args[2], "qnn.conv2d_transpose input_zero_point"))
        zw = np.asarray(_scalar(call.args[3], "qnn.conv2d_transpose kernel_zero_point"))
        a["input_zero_point"] = int(za.reshape(-1)[0])  # scalar or one element (QnnConv2DTransposeRel)
        if zw.ndim == 0 or zw.size == 1:
            a["kernel_zero_point"] = int(zw.reshape(-1)[0])
        else:
            # bias_add(int16(w), -int16(zp)) on the weight's axis 1 (legalizations.py:124-127): the
            # per-group output channel of an IOHW weight
            if a["kernel_layout"] != "IOHW" or zw.size != call.args[1].shape[1]:
                raise UnsupportedError("qnn.conv2d_transpose: a vector kernel zero point needs an IOHW kernel, one "
                                       "entry per output channel of a group")
            a["kernel_zero_point"] = 0
            consts["kernel_zero_points"] = zw.reshape(-1).astype(np.int32)
        a["input_scale"] = np.asarray(_scalar(call.args[4], "scale")).tolist()
        a["kernel_scale"] = np.asarray(_scalar(call.args[5], "scale")).tolist()
    elif op == "transpose":
        ins = _tensor_args(call, 1, names)
        if len(call.shape) > 6:
            raise UnsupportedError("transpose: up to 6-D")
    elif op == "nn.bias_add":
        ins = _tensor_args(call, 2, names)
        nd = len(call.args[0].shape)
        a["axis"] = a["axis"] if a["axis"] >= 0 else nd + a["axis"]
    elif op in ("add", "multiply", "left_shift", "right_shift"):
        lhs, rhs = call.args
        if lhs.shape != call.shape:
            raise UnsupportedError(f"{op}: the lhs must have the output shape ({lhs.shape} vs {call.shape})")
        nd, rs = len(lhs.shape), tuple(rhs.shape)
        padded = (1,) * (nd - len(rs)) + rs if len(rs) <= nd else None
        if isinstance(rhs, Constant) and rhs.data.size == 1:
            # a scalar operand (the realized graph's rounding bias, shift amounts, scales)
            ins = _tensor_args(call, 1, names)
            v = rhs.data.reshape(())
            a.update(ew=op, rhs_kind=1, relay_op=op,
                     scalar_f=float(v) if call.dtype == "float32" else 0.0,
                     scalar_i=int(v) if call.dtype != "float32" else 0)
            op = "ewise"
        elif rs == tuple(lhs.shape):
            ins = _tensor_args(call, 2, names)
            a.update(ew=op, rhs_kind=2, relay_op=op)
            op = "ewise"
        elif op == "add" and nd >= 2 and padded is not None and padded[1] == lhs.shape[1] and \
                all(d == 1 for i, d in enumerate(padded) if i != 1):
            # a per-channel vector: the same wrap-around (or float32) addition as nn.bias_add
            # along axis 1; the record keeps op "add"
            ins = _tensor_args(call, 2, names)
            a.update(axis=1, relay_op="add")
            op = "nn.bias_add"
        elif op == "multiply" and nd >= 2 and padded is not None and padded[1] == lhs.shape[1] and \
                all(d == 1 for i, d in enumerate(padded) if i != 1):
            # a per-channel multiplier (e.g. a batch norm's scale FoldScaleAxis left in place)
            ins = _tensor_args(call, 2, names)
            a.update(ew=op, rhs_kind=3, relay_op=op)
            op = "ewise"
        else:
            raise UnsupportedError(f"{op}: {lhs.shape} with {rs}: scalar, same-shape or per-channel "
                                   "operands only")
        if op == "ewise" and call.dtype not in ("float32", "int8", "int32", "int64"):
            raise UnsupportedError(f"{call.op} on {call.dtype}")
    elif op in ("round", "fixed_point_multiply"):
        ins = _tensor_args(call, 1, names)
        a.update(ew=op, rhs_kind=0, relay_op=op)
        op = "ewise"
    elif op in ("nn.conv2d", "nn.dense"):
        # nn.conv2d / nn.dense of a realized quantized graph (int8 x int8 -> int32, realize.cc:
        # 147-174, 207-235): the QNN contraction with zero zero points; float32 ones (layers the
        # quantizer skips) run on the float kernels
        ins = _tensor_args(call, 2, names)
        dts = (call.args[0].dtype, call.args[1].dtype, call.dtype)
        if dts == ("float32", "float32", "float32"):
            pass
        elif dts[0] in ("int8", "uint8") and dts[1] in ("int8", "uint8") and dts[2] == "int32":
            a.update(input_zero_point=0, kernel_zero_point=0, input_scale=1.0, kernel_scale=1.0, relay_op=op)
            op = "qnn." + op.split(".")[1]
        else:
            raise UnsupportedError(f"{op} with {dts}: float32 or int8 x int8 -> int32 only")
        if "groups" not in a and op.endswith("conv2d"):
            a["groups"] = 1
    elif op in ("tachikoma.qnn.conv2d", "tachikoma.qnn.dense"):
        # a tachikoma BYOC composite (relay/contrib/tachikoma.py): the contraction with zero
        # zero points, then the float32 post-ops whose folded constants ride in the attrs
        ins = _tensor_args(call, len(call.args), names)
        a["input_zero_point"] = 0
        a["kernel_zero_point"] = 0
        po = a.pop("postops")
        consts["postops_bias"] = np.asarray(po["bias"], np.float32).reshape(-1)
        consts["postops_o_scl"] = np.asarray(po["o_scl"], np.float32).reshape(-1)
        a.update(act_scl=float(po["act_scl"]), sum_scl=float(po["sum_scl"]), dst_zp=float(po["dst_zp"]),
                 clip_lo=float(po["clip"][0]), clip_hi=float(po["clip"][1]), has_sum=int(len(ins) > 2))
    elif op in ("clip", "nn.relu") and call.dtype == "float32":
        ins = _tensor_args(call, 1, names)
        if op == "clip":
            a.update(ew="clip", rhs_kind=0, lo=float(a["a_min"]), hi=float(a["a_max"]), relay_op=op)
        else:
            a.update(ew="relu", rhs_kind=0, relay_op=op)
        op = "ewise"
    elif op == "clip":
        ins = _tensor_args(call, 1, names)
        a["lo"] = _clip_bound(a["a_min"], call.dtype)
        a["hi"] = _clip_bound(a["a_max"], call.dtype)
    elif op == "nn.relu":
        ins = _tensor_args(call, 1, names)
        a["lo"] = 0
        a["hi"] = int(np.iinfo(np.dtype(call.dtype)).max)
    elif op == "nn.pad":
        ins = _tensor_args(call, 1, names)
        if call.dtype not in INT_DTYPES + ("float32",) or len(call.shape) > 6:
            raise UnsupportedError(f"nn.pad on {call.dtype} / {len(call.shape)}-D")
        a["value"] = call.args[1].data.item()
    elif op in ("cast", "nn.max_pool2d", "nn.avg_pool2d", "nn.global_avg_pool2d", "nn.batch_flatten", "reshape",
                "annotation.stop_fusion", "annotation.cast_hint"):
        ins = _tensor_args(call, 1, names)
        ok = INT_DTYPES + ("float32",)
        if op == "cast" and (call.args[0].dtype not in ok or call.dtype not in ok):
            raise UnsupportedError("cast: integer and float32 types only")
        if op == "nn.avg_pool2d" and call.dtype == "float32":
            raise UnsupportedError("nn.avg_pool2d: float32 is not on the device path")
        if op != "cast" and call.dtype not in ok:
            raise UnsupportedError(f"{op} on {call.dtype}")
    else:
        raise UnsupportedError(f"operator {op} is not on the integer trace path")
    return PlanOp(index, name, op, ins, a, out, consts)


@dataclass
class ExecGroup:
    """One device node: a single op, or a fused layer block
    ``qnn.conv2d|qnn.dense → nn.bias_add → qnn.requantize [→ clip|nn.relu]`` or residual join
    ``qnn.add [→ clip|nn.relu]`` whose every op output is still written (and traced) separately."""
    kind: str            # op name, "conv_block", "dense_block" or "add_block"

    @property
    def add(self) -> Optional["PlanOp"]:
        """The residual qnn.add absorbed by a conv block, if any."""
        return self.ops[3] if len(self.ops) > 3 and self.ops[3].op == "qnn.add" else None
    ops: List[PlanOp]

    @property
    def last(self) -> PlanOp:
        return self.ops[-1]


def exec_groups(plan: Plan, fuse: bool = True) -> List[ExecGroup]:
    """Group the plan's ops into device nodes.

    A chain fuses when each op is the first consumer of its predecessor's output; other
    consumers of the intermediates stay correct because every intermediate is materialised
    in its own HBM buffer anyway.  The requantize must run along the channel axis (1).

    A conv block whose requantize output feeds a same-shape 8-bit ``qnn.add`` (the ResNet
    bottleneck tail) also absorbs the add [→ clip] when nothing else reads the block's
    intermediates; that group runs at the add's position in topological order, where the
    add's other operand (the residual) is available.  Every other group runs at its
    first op's position."""
    consumers: Dict[str, List[PlanOp]] = {}
    for op in plan.ops:
        for x in op.inputs:
            consumers.setdefault(x, []).append(op)
    pos = {op.name: i for i, op in enumerate(plan.ops)}
    taken = set()
    placed: List[Tuple[int, int, ExecGroup]] = []

    def first_consumer(op: PlanOp, kind) -> Optional[PlanOp]:
        for c in consumers.get(op.name, []):
            if c.op in kind and c.inputs[0] == op.name and c.name not in taken:
                return c
        return None

    def residual_add(rq: PlanOp, chain: List[PlanOp]) -> Optional[PlanOp]:
        cs = consumers.get(rq.name, [])
        if len(cs) != 1 or cs[0].op != "qnn.add" or cs[0].name in taken:
            return None
        add = cs[0]
        if add.out.dtype != rq.out.dtype or add.inputs[0] == add.inputs[1] or not add.attrs.get("per_tensor") \
                or add.attrs.get("compute_dtype", "int64") != "int64":
            return None
        other = add.inputs[1] if add.inputs[0] == rq.name else add.inputs[0]
        if plan.tensor(other).shape != rq.out.shape or plan.tensor(other).dtype != rq.out.dtype:
            return None
        # the block's intermediates must have no reader outside the chain
        members = {c.name for c in chain} | {add.name}
        for c in chain[:-1]:
            if any(x.name not in members for x in consumers.get(c.name, [])):
                return None
        return add

    def place(at: int, group: ExecGroup):
        placed.append((at, len(placed), group))

    for op in plan.ops:
        if op.name in taken:
            continue
        nchw = op.attrs.get("data_layout", "NCHW") == "NCHW" and op.attrs.get("kernel_layout", "OIHW") == "OIHW" \
            and op.attrs.get("depthwise_multiplier", 1) == 1
        if fuse and op.op in ("qnn.conv2d", "qnn.dense") and nchw:
            b = first_consumer(op, ("nn.bias_add",))
            rq = first_consumer(b, ("qnn.requantize",)) if b is not None and b.attrs["axis"] == 1 else None
            if rq is not None and rq.out.dtype in ("int8", "uint8") and rq.attrs["channel_axis"] == 1 \
                    and b.out.dtype == "int32" and rq.attrs.get("compute_dtype", "int64") == "int64":
                chain = [op, b, rq]
                add = residual_add(rq, chain) if op.op == "qnn.conv2d" else None
                if add is not None:
                    chain.append(add)
                    cl = first_consumer(add, ("clip", "nn.relu"))
                else:
                    cl = first_consumer(rq, ("clip", "nn.relu"))
                if cl is not None:
                    chain.append(cl)
                for c in chain:
                    taken.add(c.name)
                kind = "conv_block" if op.op == "qnn.conv2d" else "dense_block"
                place(pos[add.name] if add is not None else pos[op.name], ExecGroup(kind, chain))
                continue
        if fuse and op.op == "qnn.add" and op.out.dtype in ("int8", "uint8") and op.attrs.get("per_tensor") and \
                op.attrs.get("compute_dtype", "int64") == "int64" and \
                all(plan.tensor(x).shape == op.out.shape for x in op.inputs[:2]):
            chain = [op]
            cl = first_consumer(op, ("clip", "nn.relu"))
            if cl is not None:
                chain.append(cl)
            for c in chain:
                taken.add(c.name)
            place(pos[op.name], ExecGroup("add_block", chain))
            continue
        taken.add(op.name)
        place(pos[op.name], ExecGroup(op.op, [op]))
    placed.sort(key=lambda t: (t[0], t[1]))
    return [g for _, _, g in placed]


class ExecutorFactory:
    """What ``relay.build`` returns (backend/executor_factory.py:148-211 analogue)."""

    def __init__(self, plan: Plan, params: Dict[str, np.ndarray], target: str, mod_name: str = "default",
                 fuse: bool = True):
        self.fuse = fuse
        self.plan = plan
        self.params = params
        self.target = target
        self.mod_name = mod_name

    def __getitem__(self, key: str):
        if key != self.mod_name:
            raise KeyError(key)
        return self._create

    def get_params(self) -> Dict[str, np.ndarray]:
        return dict(self.params)

    def get_graph_json(self) -> str:
        """The lowered plan as JSON (the graph-JSON role of executor_factory.py:get_graph_json)."""
        import json
        from ..runtime import plan_to_json
        return json.dumps(plan_to_json(self.plan))

    def get_executor_config(self) -> str:
        return self.get_graph_json()

    def save(self) -> bytes:
        """SaveToBinary analogue (json_runtime.h:105-135): plan + params + op constants."""
        from ..runtime import serialize_module
        return serialize_module(self)

    def export_library(self, path: str) -> str:
        """executor_factory.py:144-211 analogue: one file that ``runtime.load_module`` reloads
        without re-lowering (the kernels are the in-tree library)."""
        with open(path, "wb") as f:
            f.write(self.save())
        return path

    def _create(self, dev=None, tune=True):
        """``lib["default"](dev)``; ``tune`` as for DeviceModule (True: find step on this GPU; a tune
        table or its path: replay it)."""
        from .device_module import DeviceModule
        return DeviceModule(self.plan, self.params, dev, fuse=self.fuse, tune=tune)


def build(mod, target: str = "mi355x", params=None, mod_name: str = "default", fuse: bool = True) -> ExecutorFactory:
    t = str(target).split()[0].lower()
    if t not in TARGETS:
        raise UnsupportedError(
            f"target {target!r}: this engine builds for MI355X only ({', '.join(TARGETS)}); "
            "the reference's CPU llvm path is not part of it")
    if isinstance(params, (bytes, bytearray, memoryview)):
        # a params blob as written by save_param_dict / SaveParams (file_utils.cc:184-206)
        from ..runtime import load_param_dict
        params = load_param_dict(bytes(params))
    params = {k: np.ascontiguousarray(np.asarray(v.numpy() if hasattr(v, "numpy") else v))
              for k, v in (params or {}).items()}
    mod = _simplify_batch_norms(mod, params)
    mod, params = lift_constants(mod, params)
    plan = lower(mod, params)
    return ExecutorFactory(plan, params, t, mod_name, fuse=fuse)


def _simplify_batch_norms(mod, params: Dict[str, np.ndarray]):
    """The reference's pass prefix runs SimplifyInference + FoldConstant on every build
    (src/relay/backend/utils.cc:239-258): a graph with ``nn.batch_norm`` layers gets their
    inference form (per-channel multiply + add, relay/transform.py), the scale / shift folded to
    constants (the four statistics bound from ``params`` when they are parameters)."""
    func = mod["main"] if isinstance(mod, IRModule) else IRModule.from_expr(mod)["main"]
    bns = [n for n in post_order(func.body) if isinstance(n, Call) and n.op == "nn.batch_norm"]
    if not bns:
        return mod
    from .fold import fold_constant, rebuild
    from .transform import simplify_inference
    stats = {id(v) for n in bns for v in n.args[1:] if isinstance(v, Var) and v.name_hint in params}

    def bind(call: Call, args):
        args = [Constant(params[a.name_hint]) if id(a) in stats else a for a in args]
        return Call(call.op, args, call.attrs, call.checked_type)

    body = rebuild(func.body, bind)
    keep = [p for p in func.params if id(p) not in stats]
    return fold_constant(simplify_inference(IRModule(Function(keep, body))))


def lift_constants(mod, params: Dict[str, np.ndarray]):
    """Tensor-valued constants (the folded weights and biases of a ``relay.quantize`` result)
    become params named ``_const<k>``, uploaded once like any weight; scalar constants stay in
    the ops' attributes.  QNN ops' scale / zero-point arguments are left alone."""
    func = mod["main"] if isinstance(mod, IRModule) else IRModule.from_expr(mod)["main"]
    params = dict(params)
    lifted: Dict[int, Var] = {}

    def lift(c: Constant) -> Expr:
        if id(c) not in lifted:
            name = f"_const{len(lifted)}"
            while name in params:
                name += "_"
            lifted[id(c)] = Var(name, c.data.shape, str(c.data.dtype))
            params[name] = np.ascontiguousarray(c.data)
        return lifted[id(c)]

    new: Dict[int, Expr] = {}
    for n in post_order(func.body):
        if isinstance(n, Tuple):
            fields = [new.get(id(x), x) for x in n.fields]
            if any(x is not y for x, y in zip(fields, n.fields)):
                new[id(n)] = Tuple(fields)
            continue
        if not isinstance(n, Call):
            continue
        # tensor operands only: a QNN op's scale / zero-point arguments stay constants
        if n.op in ("qnn.requantize", "qnn.quantize", "qnn.dequantize", "qnn.concatenate", "qnn.simulated_quantize",
                    "qnn.simulated_dequantize"):
            k = 1
        elif n.op == "reshape" and isinstance(n.args[0], Constant):
            k = 0  # a reshaped constant (the simulated ops' parameters) folds in lower(), like FoldConstant
        elif n.op.startswith("qnn."):
            k = 2
        else:
            k = len(n.args)
        args = [new.get(id(x), x) for x in n.args]
        args = [lift(x) if i < k and isinstance(x, Constant) and x.data.size > 1 else x for i, x in enumerate(args)]
        if any(x is not y for x, y in zip(args, n.args)):
            new[id(n)] = Call(n.op, args, n.attrs, n.checked_type)
    if not lifted:
        return mod, params
    body = new.get(id(func.body), func.body)
    return IRModule(Function(list(func.params) + [lifted[k] for k in lifted], body)), params

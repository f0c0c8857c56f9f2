"""The reference's canonical (post-QNN-lowering) graph of a plan, for the fused-node debug dump.

The reference executor never runs QNN ops: ``relay.build``'s pass prefix (src/relay/backend/
utils.cc:222-282) first legalizes them for its target -- x86 without fast int8,
``helper_no_fast_int8_hw_legalization`` (python/tvm/relay/qnn/op/legalizations.py:177-232) -- and
canonicalizes them (FTVMQnnCanonicalize), then simplifies (SimplifyExpr, EliminateCommonSubexpr,
CanonicalizeOps) and only then fuses (FuseOps).  Its fused functions, their names
(``tvmgen_default_fused_nn_conv2d_add_fixed_point_multiply_clip_cast_cast``) and the tensors its
debug executor dumps are those of that canonical graph.  This module rebuilds it from the plan:

* ``qnn.conv2d`` / ``qnn.dense``: ``cast(data, int16)``, ``subtract(., zp)`` (legalizations.py:
  195-226), then ``nn.conv2d`` / ``nn.dense`` on int16 operands with int32 output; the weight's
  cast / zero-point shift is folded into a constant (FoldConstant);
* ``qnn.requantize``: RequantizeLowerInt (src/relay/qnn/op/requantize.cc:195-273): ``cast(int32)``,
  ``subtract`` of the input zero point, ``fixed_point_multiply`` (per tensor, UPWARD) or
  ``fixed_point_multiply_per_axis`` (per channel, FixedPointMultiplyPerChannel, qnn/utils.cc:111-135),
  ``add`` of the output zero point, ``clip`` + ``cast`` unless the output is int32;
* ``qnn.add``: QnnAddCanonicalize (src/relay/qnn/op/add.cc:40-96) -- each operand through
  RequantizeOrUpcast (op_common.h:186-200: the requantize above to int32, or a ``cast``), ``add``,
  ``subtract`` of the output zero point, ConvertDtype (``clip`` + ``cast``);
* ``nn.bias_add`` -> ``add`` (CanonicalizeOps, canonicalize_ops.cc; the bias's expand_dims folded);
* SimplifyExpr (simplify_expr.cc:700-968) on the result: EliminateIdentity (``x - 0``, ``x + 0``),
  SimplifySameCast, SimplifyConsecutiveCast (widening first casts), SimplifyClipAndConsecutiveCast
  (``clip -> cast(t) -> cast(int32)`` with t's range as bounds), SimplifyCastClip (a ``clip`` to the
  range of the preceding cast's type); EliminateCommonSubexpr merges identical calls (the shared
  int16 shift of a tensor read by two convs).

Every canonical op keeps the plan record its value equals, where there is one (the contraction,
the requantize / add / clip outputs), so that only the intermediates (int16 shifts, int32 partial
requantize results) need computing when the dump is made.  TONEAREST requantize is lowered like
the reference's FixedPointMultiplyToNearest (int64 cast, left_shift, multiply, greater_equal /
where rounding constant, add, right_shift, cast).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .build_module import UnsupportedError


@dataclass
class CTensor:
    name: str
    shape: Tuple[int, ...]
    dtype: str


@dataclass
class CanonOp:
    """One call of the canonical graph (the plan-op interface relay/fuse.py works on)."""
    name: str
    op: str
    inputs: List[str]
    attrs: Dict[str, Any]
    out: CTensor
    consts: Dict[str, np.ndarray] = field(default_factory=dict)
    origin: str = ""              # the plan (QNN-level) op it was lowered from
    record: Optional[str] = None  # plan record holding exactly this value, if any


@dataclass
class CanonPlan:
    inputs: list
    params: list
    ops: List[CanonOp]
    outputs: List[str]

    def tensor(self, name: str):
        for t in list(self.inputs) + list(self.params):
            if t.name == name:
                return t
        for o in self.ops:
            if o.name == name:
                return o.out
        raise KeyError(name)


_RANGE = {"int8": (-128, 127), "uint8": (0, 255), "int16": (-32768, 32767), "uint16": (0, 65535),
          "int32": (-2**31, 2**31 - 1)}


def _widening(src: str, dst: str) -> bool:
    """SimplifyConsecutiveCast::IsWidenCast for the integer types here (int < uint in code order)."""
    s, d = np.dtype(src), np.dtype(dst)
    if s.kind == d.kind:
        return s.itemsize <= d.itemsize
    return s.kind == "i" and d.kind == "u" and s.itemsize <= d.itemsize


class _Builder:
    def __init__(self, plan, simplify_clip_cast: bool = True):
        self.plan = plan
        self.simplify_clip_cast = simplify_clip_cast
        self.ops: List[CanonOp] = []
        self.val: Dict[str, str] = {}      # plan tensor -> canonical tensor holding its value
        self.info: Dict[str, CTensor] = {}
        for t in list(plan.inputs) + list(plan.params):
            self.val[t.name] = t.name
            self.info[t.name] = CTensor(t.name, tuple(t.shape), t.dtype)
        self.cse: Dict[str, str] = {}
        self.origin = ""
        self.k = 0

    def t(self, name: str) -> CTensor:
        return self.info[name]

    def emit(self, op: str, inputs: List[str], attrs: Dict[str, Any], shape, dtype: str,
             consts: Optional[Dict[str, np.ndarray]] = None) -> str:
        consts = consts or {}
        key = repr((op, inputs, sorted(attrs.items()), dtype,
                    [(k, v.dtype.str, v.shape, v.tobytes()) for k, v in sorted(consts.items())]))
        if key in self.cse:  # EliminateCommonSubexpr
            return self.cse[key]
        name = f"{self.origin}.c{self.k}"
        self.k += 1
        c = CanonOp(name, op, list(inputs), dict(attrs), CTensor(name, tuple(shape), dtype), dict(consts), self.origin)
        self.ops.append(c)
        self.info[name] = c.out
        self.cse[key] = name
        return name

    # ---- elementary ops with the SimplifyExpr rewrites applied as they are formed
    def cast(self, x: str, dtype: str) -> str:
        t = self.t(x)
        if t.dtype == dtype:  # SimplifySameCast
            return x
        prod = self._producer(x)
        if prod is not None and prod.op == "cast":
            src = self.t(prod.inputs[0])
            if _widening(src.dtype, t.dtype):  # SimplifyConsecutiveCast
                return self.cast(prod.inputs[0], dtype)
            clip = self._producer(prod.inputs[0])
            if self.simplify_clip_cast and clip is not None and clip.op == "clip" and clip.out.dtype == dtype and \
                    (clip.attrs["a_min"], clip.attrs["a_max"]) == _RANGE.get(t.dtype):
                return clip.name  # SimplifyClipAndConsecutiveCast
        return self.emit("cast", [x], {"dtype": dtype}, t.shape, dtype)

    def clip(self, x: str, lo: int, hi: int) -> str:
        t = self.t(x)
        prod = self._producer(x)
        if prod is not None and prod.op == "cast" and (lo, hi) == _RANGE.get(t.dtype):
            return x  # SimplifyCastClip
        return self.emit("clip", [x], {"a_min": int(lo), "a_max": int(hi)}, t.shape, t.dtype)

    def subtract_scalar(self, x: str, v: int) -> str:
        if int(v) == 0:  # EliminateIdentity
            return x
        t = self.t(x)
        return self.emit("subtract", [x], {"scalar": int(v)}, t.shape, t.dtype)

    def add_scalar(self, x: str, v: int) -> str:
        if int(v) == 0:
            return x
        t = self.t(x)
        return self.emit("add", [x], {"scalar": int(v)}, t.shape, t.dtype)

    def _producer(self, name: str) -> Optional[CanonOp]:
        for o in reversed(self.ops):
            if o.name == name:
                return o
        return None

    # ---- QNN lowerings
    def requantize_lower(self, x: str, attrs: Dict[str, Any], consts: Dict[str, np.ndarray], axis: int,
                         out_dtype: str) -> str:
        """RequantizeLowerInt (requantize.cc:195-273) on canonical tensor x."""
        t = self.cast(x, "int32")
        if "input_zero_points" in consts:
            zp = consts["input_zero_points"]
            t = self.emit("subtract", [t], {"axis": axis}, self.t(t).shape, "int32",
                          {"vector": np.asarray(zp, np.int32)}) if np.any(zp) else t
        else:
            t = self.subtract_scalar(t, attrs.get("input_zero_point", 0))
        if attrs.get("rounding", "UPWARD") == "TONEAREST":
            if "multipliers" in consts:
                t = self.to_nearest(t, np.asarray(consts["multipliers"]), np.asarray(consts["shifts"]), axis)
            elif attrs.get("mode", 3) != 0:
                t = self.to_nearest(t, np.array([attrs["multiplier"]]), np.array([attrs["shift"]]), None)
        elif "multipliers" in consts:
            t = self.emit("fixed_point_multiply_per_axis", [t], {"axis": axis}, self.t(t).shape, "int32",
                          {"multipliers": consts["multipliers"], "shifts": consts["shifts"]})
        elif attrs.get("mode", 2) != 0:  # identity: equal scales skip the multiply (requantize.cc:226)
            if attrs.get("mode") == 1:  # power of two: tir.q_multiply_shift with m = 2^30
                t = self.emit("fixed_point_multiply", [t], {"multiplier": 1 << 30, "shift": int(attrs["shift"])},
                              self.t(t).shape, "int32")
            else:
                t = self.emit("fixed_point_multiply", [t], {"multiplier": int(attrs["multiplier"]),
                                                            "shift": int(attrs["shift"])}, self.t(t).shape, "int32")
        t = self.add_scalar(t, attrs.get("output_zero_point", 0))
        if out_dtype != "int32":
            lo, hi = _RANGE[out_dtype]
            t = self.cast(self.clip(t, lo, hi), out_dtype)
        return t

    def to_nearest(self, t: str, ms: np.ndarray, ss: np.ndarray, axis: Optional[int]) -> str:
        """FixedPointMultiplyToNearest (src/relay/qnn/utils.cc:59-109; per channel :137-216, axis not
        None): in int64, [left_shift], multiply, add where(x >= 0, 2^(30+rs), 2^(30+rs) - 1),
        right_shift by 31 + rs, cast to int32.  The zeros / full / broadcast_to operands are constants
        after FoldConstant."""
        shape = self.t(t).shape
        ls = np.maximum(ss, 0).astype(np.int64)
        rs = np.maximum(-ss, 0).astype(np.int64)
        total = rs + 31
        pos = (np.int64(1) << (total - 1)).astype(np.int64)
        x = self.cast(t, "int64")

        def operand(v: np.ndarray):
            # scalar constant (per-tensor) or an axis-expanded vector (per-channel)
            return ({"scalar": int(v[0])}, {}) if axis is None else ({"axis": axis}, {"vector": v.astype(np.int64)})

        if np.any(ls):
            a, c = operand(ls)
            x = self.emit("left_shift", [x], a, shape, "int64", c)
        a, c = operand(np.asarray(ms, np.int64))
        x = self.emit("multiply", [x], a, shape, "int64", c)
        ge = self.emit("greater_equal", [x], {"scalar": 0}, shape, "bool")
        wa = {} if axis is None else {"axis": axis}
        r = self.emit("where", [ge], wa, shape, "int64", {"pos": pos, "neg": pos - 1})
        x = self.emit("add", [x, r], {}, shape, "int64")
        a, c = operand(total)
        x = self.emit("right_shift", [x], a, shape, "int64", c)
        return self.cast(x, "int32")

    def lower(self, p) -> None:
        self.origin, self.k = p.name, 0
        a = p.attrs
        if a.get("compute_dtype", "int64") != "int64":
            # RequantizeLowerFP's float op sequence (requantize.cc:293-373) is not restated here
            from .build_module import UnsupportedError
            raise UnsupportedError(f"canonical dump of {p.op} under compute_dtype={a['compute_dtype']}")
        ins = [self.val[x] for x in p.inputs]
        if p.op in ("qnn.conv2d", "qnn.dense"):
            d = self.subtract_scalar(self.cast(ins[0], "int16"), a["input_zero_point"])
            kind = "nn.conv2d" if p.op == "qnn.conv2d" else "nn.dense"
            keep = {k: v for k, v in a.items() if k not in ("input_zero_point", "kernel_zero_point", "input_scale",
                                                            "kernel_scale", "relay_op")}
            # the weight operand: int16(w) - zp_w folded to a constant (the plan's weight param)
            out = self.emit(kind, [d, p.inputs[1]], keep, p.out.shape, "int32",
                            {"kernel_zero_point": np.asarray(a.get("kernel_zero_point", 0), np.int32),
                             **{k: v for k, v in p.consts.items() if k == "kernel_zero_points"}})
        elif p.op == "nn.bias_add":
            ax = a["axis"]
            out = self.emit("add", [ins[0], p.inputs[1]], {"axis": ax}, p.out.shape, p.out.dtype)
        elif p.op == "qnn.requantize":
            out = self.requantize_lower(ins[0], a, p.consts, a.get("channel_axis", 1), p.out.dtype)
        elif p.op == "qnn.add":
            if not (tuple(self.t(ins[0]).shape) == tuple(self.t(ins[1]).shape) == tuple(p.out.shape)):
                # QnnBroadcastRel operands: the canonical evaluators (oracle and device) add
                # same-shape tensors only
                raise UnsupportedError(f"canonical graph: broadcasting qnn.add {p.name}")
            sides = []
            for side, x in (("lhs", ins[0]), ("rhs", ins[1])):
                if a[f"{side}_upcast"]:
                    sides.append(self.cast(x, "int32"))
                else:
                    # RequantizeOrUpcast (op_common.h:186-207): the side's Requantize with the
                    # op's rounding (requantize_config at construction) and, per axis, the side's
                    # multipliers / shifts / zero points along {side}_axis
                    ra = {"mode": a[f"{side}_mode"], "multiplier": a[f"{side}_multiplier"], "shift": a[f"{side}_shift"],
                          "input_zero_point": a[f"{side}_zero_point"], "output_zero_point": a["output_zero_point"],
                          "rounding": a.get("rounding", "UPWARD")}
                    consts = {}
                    if f"{side}_multipliers" in p.consts:
                        consts["multipliers"] = p.consts[f"{side}_multipliers"]
                        consts["shifts"] = p.consts[f"{side}_shifts"]
                    if f"{side}_zero_points" in p.consts:
                        consts["input_zero_points"] = p.consts[f"{side}_zero_points"]
                    sides.append(self.requantize_lower(x, ra, consts, a.get(f"{side}_axis", 1), "int32"))
            o = self.emit("add", sides, {}, p.out.shape, "int32")
            o = self.subtract_scalar(o, a["output_zero_point"])
            lo, hi = _RANGE[p.out.dtype]
            out = self.cast(self.clip(o, lo, hi), p.out.dtype)
        elif p.op in ("clip", "nn.relu"):
            out = self.clip(ins[0], int(a["lo"]), int(a["hi"])) if p.op == "clip" else \
                self.emit("nn.relu", [ins[0]], {}, p.out.shape, p.out.dtype)
        elif p.op == "cast":
            out = self.cast(ins[0], p.out.dtype)
        elif p.op in ("nn.max_pool2d", "nn.avg_pool2d", "nn.global_avg_pool2d", "nn.batch_flatten", "reshape"):
            out = self.emit(p.op, ins, dict(a), p.out.shape, p.out.dtype)
        else:
            raise UnsupportedError(f"canonical graph: {p.op} is not a QNN-path op")
        self.val[p.name] = out
        prod = self._producer(out)
        if prod is not None and prod.record is None and tuple(prod.out.shape) == tuple(p.out.shape) and \
                prod.out.dtype == p.out.dtype:
            prod.record = p.name


def canonicalize(plan, simplify_clip_cast: bool = True) -> CanonPlan:
    """The canonical graph of a built plan (see the module docstring).  ``simplify_clip_cast=False``
    leaves out SimplifyClipAndConsecutiveCast (what older reference builds did, see
    tests/test_canonical.py)."""
    b = _Builder(plan, simplify_clip_cast)
    for p in plan.ops:
        b.lower(p)
    outputs = [b.val[o] for o in plan.outputs]
    used = set(outputs)
    for o in b.ops:
        used.update(o.inputs)
    # ops whose result nothing reads (a cast the simplifications routed around) are dropped,
    # as dead code is by the reference's passes
    ops = [o for o in b.ops if o.name in used]
    while len(ops) != len(b.ops):
        b.ops = ops
        used = set(outputs)
        for o in ops:
            used.update(o.inputs)
        ops = [o for o in ops if o.name in used]
    return CanonPlan(list(plan.inputs), list(plan.params), ops, outputs)

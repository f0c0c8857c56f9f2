"""Device values of the canonical graph's tensors (tachikoma_amd/relay/canonical.py) for the
debug executor's ``granularity="canonical"`` dump.

A canonical op that stands for a plan record (the contraction, the bias add, the requantize /
add / clip results) is that record's device buffer; the others -- the int16 zero-point shifts
of a conv operand, the int32 partial results of a lowered requantize or qnn.add -- are computed
on the device from their canonical inputs with the C-ABI's elementwise kernels:

  cast -> tk_cast; subtract / add of a scalar -> tk_ewise (add, int16 / int32, wrapping);
  add / subtract of a per-channel vector -> tk_bias_add; add of two tensors -> tk_ewise
  (rhs_kind 2); fixed_point_multiply -> tk_ewise; fixed_point_multiply_per_axis -> tk_ewise
  (rhs_kind 3, multipliers then shifts); clip -> tk_clip; nn.relu -> tk_ewise.

There is no host path: an op outside this list raises."""
from __future__ import annotations

import ctypes
from typing import Dict

import numpy as np

from ... import _lib


class CanonicalValues:
    def __init__(self, module, canon):
        self.module = module
        self.canon = canon
        self.ops = {o.name: o for o in canon.ops}
        self._vals: Dict[str, object] = {}
        self._keep = []

    def _torch(self):
        import torch
        return torch

    def _ref(self, t) -> _lib.TensorRef:
        r = _lib.TensorRef.from_torch(t)
        self._keep.append(r)
        return r

    def _empty(self, op):
        from ...relay.device_module import torch_dtype
        return self._torch().empty(tuple(op.out.shape), dtype=torch_dtype(op.out.dtype), device=self.module.device)

    def _i32(self, arr):
        t = self._torch().from_numpy(np.ascontiguousarray(arr, dtype=np.int32)).to(self.module.device)
        self._keep.append(t)
        return t

    def _ewise(self, x, rhs, out, op: str, rhs_kind: int, scalar: int = 0, multiplier: int = 0, shift: int = 0):
        a = _lib.tk_ewise_attrs()
        a.op = _lib.TK_EW[op]
        a.rhs_kind = rhs_kind
        a.scalar_i = int(scalar)
        a.multiplier, a.shift = int(multiplier), int(shift)
        rr = self._ref(rhs).ptr if rhs is not None else None
        _lib.check(self.module.lib.tk_ewise(self._ref(x).ptr, rr, self._ref(out).ptr, ctypes.byref(a), self._stream()))

    def _stream(self):
        return ctypes.c_void_p(_lib.stream_handle(self._torch().cuda.current_stream(self.module.device)))

    def value(self, name: str):
        """Device tensor holding canonical tensor ``name`` (a plan input / param, or an op)."""
        if name in self._vals:
            return self._vals[name]
        op = self.ops.get(name)
        if op is None:
            v = self.module.buffers[name]  # plan input or param
        elif op.record is not None:
            v = self.module.buffers[op.record]
        else:
            v = self._compute(op)
        self._vals[name] = v
        return v

    def _compute(self, op):
        lib = self.module.lib
        args = [self.value(x) for x in op.inputs]
        out = self._empty(op)
        a = op.attrs
        x = args[0]
        s = self._stream()
        if op.op == "cast":
            _lib.check(lib.tk_cast(self._ref(x).ptr, self._ref(out).ptr, s))
        elif op.op in ("subtract", "add") and "scalar" in a:
            v = int(a["scalar"])
            self._ewise(x, None, out, "add", 1, scalar=-v if op.op == "subtract" else v)
        elif op.op == "subtract" and "vector" in op.consts:
            vec = self._i32(-np.asarray(op.consts["vector"], np.int64))
            _lib.check(lib.tk_bias_add(self._ref(x).ptr, self._ref(vec).ptr, self._ref(out).ptr, int(a["axis"]) % x.dim(), s))
        elif op.op == "add" and len(args) == 2:
            y = args[1]
            if tuple(y.shape) == tuple(x.shape):
                self._ewise(x, y, out, "add", 2)
            else:
                _lib.check(lib.tk_bias_add(self._ref(x).ptr, self._ref(y.reshape(-1)).ptr, self._ref(out).ptr,
                                           int(a.get("axis", 1)) % x.dim(), s))
        elif op.op == "fixed_point_multiply":
            self._ewise(x, None, out, "fixed_point_multiply", 0, multiplier=a["multiplier"], shift=a["shift"])
        elif op.op == "fixed_point_multiply_per_axis":
            if int(a["axis"]) % x.dim() != 1:
                raise _lib.TachikomaError("fixed_point_multiply_per_axis: axis 1 only")
            ms = self._i32(np.concatenate([np.asarray(op.consts["multipliers"]).reshape(-1),
                                           np.asarray(op.consts["shifts"]).reshape(-1)]))
            self._ewise(x, ms, out, "fixed_point_multiply", 3)
        elif op.op == "clip":
            _lib.check(lib.tk_clip(self._ref(x).ptr, self._ref(out).ptr, int(a["a_min"]), int(a["a_max"]), s))
        elif op.op == "nn.relu":
            self._ewise(x, None, out, "relu", 0)
        else:
            raise _lib.TachikomaError(f"canonical dump: no device evaluation for {op.op} ({op.name}) without a record")
        return out

"""Minimal Relay-style expression IR for integer QNN graphs.

Mirrors the subset of ``tvm.relay`` the reference's trace path consumes
(``python/tvm/relay/expr.py`` Var/Constant/Call, ``python/tvm/ir/module.py``
IRModule) — enough to write the same graph-building code as the reference's
tests and MRT driver, with eager type inference on construction.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np


@dataclass(frozen=True)
class TensorType:
    shape: Tuple[int, ...]
    dtype: str

    @property
    def concrete_shape(self):
        return self.shape


class Expr:
    checked_type: TensorType

    @property
    def shape(self) -> Tuple[int, ...]:
        return self.checked_type.shape

    @property
    def dtype(self) -> str:
        return self.checked_type.dtype


class Var(Expr):
    def __init__(self, name_hint: str, shape: Sequence[int], dtype: str = "float32"):
        self.name_hint = name_hint
        self.checked_type = TensorType(tuple(int(s) for s in shape), str(np.dtype(dtype)))

    def __repr__(self):
        return f"%{self.name_hint}: Tensor[{self.shape}, {self.dtype}]"


class Constant(Expr):
    def __init__(self, data: np.ndarray):
        self.data = np.asarray(data)
        self.checked_type = TensorType(tuple(self.data.shape), str(self.data.dtype))

    def is_scalar(self) -> bool:
        return self.data.ndim == 0

    def numpy(self) -> np.ndarray:
        return self.data

    def __repr__(self):
        return f"const({self.data.tolist()}, {self.dtype})"


class Call(Expr):
    def __init__(self, op: str, args: List[Expr], attrs: Dict[str, Any], ret: TensorType):
        self.op = op
        self.args = list(args)
        self.attrs = dict(attrs)
        self.checked_type = ret

    def __repr__(self):
        return f"{self.op}({', '.join(type(a).__name__ for a in self.args)})"


class Tuple(Expr):
    """``relay.Tuple`` (python/tvm/relay/expr.py): the tensor list of ``qnn.concatenate`` and the
    scale / zero-point tuples beside it.  It is no op: it has no record and takes no ``%N`` name
    (MRT's ``expr2symbol`` names only Calls and TupleGetItems, python/tvm/mrt/symbol.py:212-253)."""

    def __init__(self, fields: Sequence[Expr]):
        self.fields = list(fields)
        self.checked_type = TensorType((len(self.fields),), "tuple")

    @property
    def args(self) -> List[Expr]:
        return self.fields

    def __len__(self):
        return len(self.fields)

    def __getitem__(self, i: int) -> Expr:
        return self.fields[i]

    def __repr__(self):
        return f"({', '.join(type(f).__name__ for f in self.fields)})"


class Function:
    def __init__(self, params: List[Var], body: Expr):
        self.params = list(params)
        self.body = body


class IRModule:
    def __init__(self, main: Function, functions: Optional[Dict[str, Function]] = None):
        """``functions``: further global functions beside ``main`` (relay.quantize's
        partition_conversions adds quantize_inputs / quantized_main / dequantize_outputs)."""
        self.functions = dict(functions or {})
        self.functions["main"] = main

    def get_global_vars(self) -> List[str]:
        return list(self.functions)

    @staticmethod
    def from_expr(expr) -> "IRModule":
        if isinstance(expr, Function):
            return IRModule(expr)
        return IRModule(Function(free_vars(expr), expr))

    def __getitem__(self, name: str) -> Function:
        return self.functions[name]

    def astext(self, show_meta_data: bool = True) -> str:
        """Relay text (IRModule.astext); parse it back with ``relay.parse``."""
        from .parser import astext
        return astext(self, show_meta_data)


def var(name_hint: str, shape: Sequence[int] = (), dtype: str = "float32") -> Var:
    return Var(name_hint, shape, dtype)


def const(value, dtype: Optional[str] = None) -> Constant:
    """``relay.const``: python floats default to float32, ints to int32 (python/tvm/relay/expr.py)."""
    if isinstance(value, Constant):
        return value
    if dtype is None:
        if isinstance(value, float):
            dtype = "float32"
        elif isinstance(value, (bool, np.bool_)):
            dtype = "bool"
        elif isinstance(value, int):
            dtype = "int32"
    arr = np.asarray(value)
    if dtype is not None:
        arr = arr.astype(dtype)
    elif arr.dtype == np.float64:
        arr = arr.astype(np.float32)
    elif arr.dtype == np.int64:
        arr = arr.astype(np.int32)
    return Constant(arr)


def post_order(expr: Expr) -> List[Expr]:
    """Post-order DFS over args (``relay.analysis.post_order_visit``); each node once (a Tuple's
    fields are its args)."""
    out: List[Expr] = []
    seen = set()
    stack = [(expr, False)]
    while stack:
        node, expanded = stack.pop()
        if id(node) in seen:
            continue
        if expanded or not isinstance(node, (Call, Tuple)):
            seen.add(id(node))
            out.append(node)
            continue
        stack.append((node, True))
        for a in reversed(node.args):
            if id(a) not in seen:
                stack.append((a, False))
    return out


def free_vars(expr: Expr) -> List[Var]:
    return [n for n in post_order(expr) if isinstance(n, Var)]

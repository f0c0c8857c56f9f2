"""Quantization configuration (python/tvm/relay/quantize/quantize.py:37-216).

Same field names and defaults as the reference's ``QConfig._node_defaults``; ``qconfig(**kw)``
is a context manager (``with qconfig(global_scale=8.0): ...``)."""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import List, Optional


class QAnnotateKind:
    """src/relay/quantize/quantize.h:39."""
    IDENTITY = 0
    INPUT = 1
    WEIGHT = 2
    ACTIVATION = 3


_KIND_NAME = {QAnnotateKind.INPUT: "input", QAnnotateKind.WEIGHT: "weight", QAnnotateKind.ACTIVATION: "activation"}


@dataclass(frozen=True)
class QConfig:
    nbit_input: int = 8
    nbit_weight: int = 8
    nbit_activation: int = 32
    dtype_input: str = "int8"
    dtype_weight: str = "int8"
    dtype_activation: str = "int32"
    calibrate_mode: str = "global_scale"
    global_scale: float = 8.0
    weight_scale: str = "power2"
    skip_dense_layer: bool = True
    skip_conv_layers: Optional[List[int]] = field(default_factory=lambda: [0])
    do_simulation: bool = False
    round_for_shift: bool = True
    debug_enabled_ops: Optional[List[str]] = None
    rounding: str = "UPWARD"
    calibrate_chunk_by: int = -1
    partition_conversions: str = "disabled"

    def guard(self, op_name: str) -> bool:
        return self.debug_enabled_ops is None or op_name in self.debug_enabled_ops

    def get_nbit_by_kind(self, kind: int) -> int:
        return getattr(self, "nbit_" + _KIND_NAME[kind])

    def get_dtype_by_kind(self, kind: int) -> str:
        return getattr(self, "dtype_" + _KIND_NAME[kind])

    def __enter__(self):
        _STACK.append(self)
        return self

    def __exit__(self, *exc):
        _STACK.pop()


_STACK: List[QConfig] = []


def current_qconfig() -> QConfig:
    return _STACK[-1] if _STACK else QConfig()


def qconfig(**kwargs) -> QConfig:
    unknown = set(kwargs) - set(QConfig.__dataclass_fields__)
    if unknown:
        raise AttributeError(f"qconfig: unknown fields {sorted(unknown)}")
    if "skip_conv_layers" in kwargs and kwargs["skip_conv_layers"] is not None:
        kwargs["skip_conv_layers"] = [int(x) for x in kwargs["skip_conv_layers"]]
    return replace(QConfig(), **kwargs)

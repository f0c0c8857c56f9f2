"""tachikoma_amd — MI355X-native integer inference-and-trace engine.

Drop-in for the CPU per-op trace path of CortexFoundation/tachikoma (a TVM
0.11.dev0 fork): Relay-style QNN graphs are executed op by op by hand-written
gfx950 HIP kernels behind a C ABI (include/tachikoma.h) and every op output is
recorded into the tachikoma trace binary.
"""
from __future__ import annotations

from dataclasses import dataclass

__version__ = "0.1.0"


@dataclass(frozen=True)
class Device:
    device_type: str
    device_id: int = 0


def rocm(dev_id: int = 0) -> Device:
    return Device("rocm", dev_id)


def cpu(dev_id: int = 0) -> Device:
    return Device("cpu", dev_id)


from . import relay  # noqa: E402,F401
from . import contrib  # noqa: E402,F401
from . import trace_format  # noqa: E402,F401
from . import runtime  # noqa: E402,F401  (save_param_dict / load_param_dict / load_module)
from ._lib import TachikomaError  # noqa: E402,F401

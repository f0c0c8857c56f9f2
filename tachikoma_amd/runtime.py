"""Module and param serialisation: the ``tvm.runtime`` surface this path needs.

* ``save_param_dict`` / ``load_param_dict`` — python/tvm/runtime/params.py:22-69
  (``SaveParams`` / ``LoadParams``, src/runtime/file_utils.cc:184-236): the NDArray-list
  blob, written through the C ABI (tk_ndlist_layout / tk_ndlist_write_headers).
* ``ExecutorFactory.export_library(path)`` → ``load_module(path)`` — the analogue of
  ``export_library`` (python/tvm/relay/backend/executor_factory.py:144-211) and of the JSON
  runtime's ``SaveToBinary`` / ``LoadFromBinary`` (src/runtime/contrib/json/json_runtime.h:
  105-135), which store the graph JSON plus the constants.  A built module here is a lowered
  ``Plan`` (ops with their folded QNN constants, MRT names) plus its params; the kernels are
  the in-tree library, so nothing else needs storing.  Reloading skips parsing and lowering
  and creates the device module directly.

Module file (little-endian)::

    u64 "TKMODULE" | u64 version | u64 json_len | u64 blob_off | u64 blob_size
    json   {"format", "version", "target", "mod_name", "fuse", "plan": {...}}
    pad to 64
    blob   NDArray-list: the params by name, then every op constant as "%const/<op>/<key>"
"""
from __future__ import annotations

import json
import struct
from typing import Any, Dict

import numpy as np

from . import trace_format as tf

MODULE_MAGIC = int.from_bytes(b"TKMODULE", "little")
MODULE_VERSION = 1
_HDR = struct.Struct("<5Q")
_CONST = "%const/"


def save_param_dict(params: Dict[str, Any]) -> bytes:
    """python/tvm/runtime/params.py:save_param_dict."""
    arrs = {k: np.ascontiguousarray(np.asarray(v.numpy() if hasattr(v, "numpy") else v)) for k, v in params.items()}
    return tf.save_ndarray_list(arrs)


def load_param_dict(param_bytes) -> Dict[str, np.ndarray]:
    """python/tvm/runtime/params.py:load_param_dict (arrays are copies)."""
    if isinstance(param_bytes, str):
        with open(param_bytes, "rb") as f:
            param_bytes = f.read()
    return tf.parse_ndarray_list(bytes(param_bytes), copy=True)


def _py(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.integer):
        return int(v)
    if isinstance(v, np.floating):
        return float(v)
    if isinstance(v, np.bool_):
        return bool(v)
    if isinstance(v, tuple):
        return [_py(x) for x in v]
    if isinstance(v, list):
        return [_py(x) for x in v]
    if isinstance(v, dict):
        return {k: _py(x) for k, x in v.items()}
    return v


def plan_to_json(plan) -> Dict[str, Any]:
    def t(x):
        return {"name": x.name, "shape": list(x.shape), "dtype": x.dtype}
    return {"inputs": [t(x) for x in plan.inputs], "params": [t(x) for x in plan.params],
            "outputs": list(plan.outputs),
            "ops": [{"index": o.index, "name": o.name, "op": o.op, "inputs": list(o.inputs),
                     "attrs": _py(o.attrs), "out": t(o.out), "consts": sorted(o.consts)} for o in plan.ops]}


def plan_from_json(doc: Dict[str, Any], consts: Dict[str, np.ndarray]):
    from .relay.build_module import Plan, PlanOp, PlanTensor

    def t(x):
        return PlanTensor(x["name"], tuple(int(s) for s in x["shape"]), x["dtype"])
    ops = []
    for o in doc["ops"]:
        cs = {k: consts[f"{_CONST}{o['name']}/{k}"] for k in o["consts"]}
        ops.append(PlanOp(o["index"], o["name"], o["op"], list(o["inputs"]), dict(o["attrs"]), t(o["out"]), cs))
    return Plan([t(x) for x in doc["inputs"]], [t(x) for x in doc["params"]], ops, list(doc["outputs"]))


def serialize_module(factory) -> bytes:
    """SaveToBinary analogue of a built module (see the module docstring)."""
    plan = factory.plan
    doc = {"format": "tachikoma-module", "version": MODULE_VERSION, "target": factory.target,
           "mod_name": factory.mod_name, "fuse": bool(factory.fuse), "plan": plan_to_json(plan)}
    arrs: Dict[str, np.ndarray] = {}
    for p in plan.params:
        arrs[p.name] = np.ascontiguousarray(factory.params[p.name])
    for o in plan.ops:
        for k, v in o.consts.items():
            arrs[f"{_CONST}{o.name}/{k}"] = np.ascontiguousarray(v)
    blob = tf.save_ndarray_list(arrs)
    text = json.dumps(doc, separators=(",", ":")).encode()
    off = (_HDR.size + len(text) + 63) // 64 * 64
    head = _HDR.pack(MODULE_MAGIC, MODULE_VERSION, len(text), off, len(blob))
    return head + text + b"\0" * (off - _HDR.size - len(text)) + blob


def deserialize_module(data: bytes):
    """LoadFromBinary analogue: returns the ``ExecutorFactory`` (``lib["default"](dev)``)."""
    from .relay.build_module import ExecutorFactory
    if len(data) < _HDR.size:
        raise ValueError("truncated tachikoma module")
    magic, version, jl, off, size = _HDR.unpack_from(data, 0)
    if magic != MODULE_MAGIC:
        raise ValueError("not a tachikoma module (bad magic)")
    if version != MODULE_VERSION:
        raise ValueError(f"unsupported tachikoma module version {version}")
    if off + size > len(data) or _HDR.size + jl > off:
        raise ValueError("truncated tachikoma module")
    doc = json.loads(bytes(data[_HDR.size:_HDR.size + jl]).decode())
    arrs = tf.parse_ndarray_list(data, off, size, copy=True)
    plan = plan_from_json(doc["plan"], arrs)
    params = {p.name: arrs[p.name] for p in plan.params}
    return ExecutorFactory(plan, params, doc["target"], doc["mod_name"], fuse=doc["fuse"])


def load_module(path: str):
    """tvm.runtime.load_module analogue for a file written by ``export_library``."""
    with open(path, "rb") as f:
        return deserialize_module(f.read())

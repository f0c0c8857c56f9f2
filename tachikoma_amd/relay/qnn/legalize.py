"""Table-lookup legalization of the qnn unary ops (python/tvm/relay/qnn/op/legalizations.py:54-86,
canonicalizations.py:32-160).

The reference builds, when it legalizes the graph, a table holding the op's result for every bit
pattern of the 8-bit input: the patterns are dequantized (qnn.dequantize, float32), mapped through
the op's numpy function and quantized back (qnn.quantize); the graph then runs
``take(table, reinterpret(x, uint8))``.  Here the table is built the same way when the device module
is created -- qnn.dequantize and qnn.quantize are this library's bit-exact kernels
(tk_qnn_dequantize / tk_qnn_quantize), the float functions are the ones the reference registers --
and the node runs tk_qnn_lookup.  The tables depend on numpy's (and scipy's) float32
implementations of these functions, as the reference's do: bit parity with a reference build is
pinned only by its tests' goldens (tests/golden/qnn_kats.json, test_op_qnn_unary_elementwise.py).
"""
from __future__ import annotations

import ctypes

import numpy as np


def _hardswish(x):
    # hardswish_func (legalizations.py:70-73)
    x2 = x + 3.0
    x2 = np.clip(x2, 0.0, 6.0)
    return x * x2 / 6.0


def _erf(x):
    from scipy import special
    return special.erf(x)


# register_qnn_unary_op_legalize calls (legalizations.py:78-86)
FUNCTIONS = {
    "qnn.sqrt": np.sqrt,
    "qnn.rsqrt": lambda arr: 1 / np.sqrt(arr),
    "qnn.exp": np.exp,
    "qnn.erf": _erf,
    "qnn.sigmoid": lambda arr: 1 / (1 + np.exp(-arr)),
    "qnn.hardswish": _hardswish,
    "qnn.tanh": np.tanh,
    "qnn.log": np.log,
    "qnn.abs": np.abs,
}


def build_table(lib, op: str, dtype: str, in_scale: float, in_zero_point: int, out_scale: float,
                out_zero_point: int, device, stream: int):
    """The op's 256-entry table as a device uint8 tensor (create_integer_lookup_table): entry i is
    the result for the input whose bit pattern is i."""
    import torch

    from ... import _lib
    from ..device_module import torch_dtype
    bits = torch.arange(256, dtype=torch.int32).to(torch.uint8).view(torch_dtype(dtype)).to(device)
    deq = torch.empty(256, dtype=torch.float32, device=device)
    keep = [_lib.TensorRef.from_torch(t) for t in (bits, deq)]
    qa = _lib.tk_qparams_attrs()
    qa.axis, qa.scale, qa.zero_point = -1, float(in_scale), int(in_zero_point)
    _lib.check(lib.tk_qnn_dequantize(keep[0].ptr, keep[1].ptr, ctypes.byref(qa), ctypes.c_void_p(stream)),
               f"{op} table: dequantize")
    torch.cuda.current_stream(device).synchronize()
    with np.errstate(all="ignore"):
        f = np.asarray(FUNCTIONS[op](deq.cpu().numpy()))
    if f.dtype != np.float32:
        # qnn.quantize takes float32 (QuantizeRel); every registered function keeps float32
        raise TypeError(f"{op}: the float function returned {f.dtype}")
    fin = torch.from_numpy(np.ascontiguousarray(f)).to(device)
    out = torch.empty(256, dtype=torch_dtype(dtype), device=device)
    refs = [_lib.TensorRef.from_torch(t) for t in (fin, out)]
    qo = _lib.tk_qparams_attrs()
    qo.axis, qo.scale, qo.zero_point = -1, float(out_scale), int(out_zero_point)
    _lib.check(lib.tk_qnn_quantize(refs[0].ptr, refs[1].ptr, ctypes.byref(qo), ctypes.c_void_p(stream)),
               f"{op} table: quantize")
    torch.cuda.current_stream(device).synchronize()
    return out.view(torch.uint8)

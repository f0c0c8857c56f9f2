"""Per-op record-and-run over a Relay-style QNN graph on the CPU (TEST INFRASTRUCTURE ONLY).

Restates ``mrt.Trace.calibrate`` (python/tvm/mrt/trace.py:65-117): walk the graph
in topological order, execute every op in isolation on its arguments' recorded
outputs, record ``outputs[name] = op(*args)``.  Symbol names follow MRT's
``expr2symbol`` (python/tvm/mrt/symbol.py:212-253): variables keep their
``name_hint``; calls are named ``%0, %1, ...`` in post-order.  Each op's
arithmetic comes from oracle/qnn_ref.py (numpy) or, for conv/dense, the OpenMP C
restatement oracle/qnn_ref.c (identical semantics, used for large inputs).

This walker re-implements the traversal and constant folding independently of
``tachikoma_amd.relay.build_module`` so it can check the product's lowering.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import numpy as np

from . import qnn_ref as ref


def _post_order(expr):
    out, seen = [], set()

    def visit(node):
        if id(node) in seen:
            return
        for a in getattr(node, "args", []):
            visit(a)
        seen.add(id(node))
        out.append(node)

    import sys
    sys.setrecursionlimit(max(10000, sys.getrecursionlimit()))
    visit(expr)
    return out


def _const(e):
    assert type(e).__name__ == "Constant", f"expected a constant, got {type(e).__name__}"
    return e.data


def _pad4(p):
    p = tuple(int(v) for v in p)
    return p if len(p) == 4 else (p[0], p[1], p[0], p[1])


def _conv_c(x, w, za, zw, a, threads):
    from . import c_lib
    lib = c_lib()
    n, c, h, wd = x.shape
    o, cg, kh, kw = w.shape
    sh, sw = a["strides"]
    dh, dw = a["dilation"]
    pt, pl, pb, pr = _pad4(a["padding"])
    oh = (h + pt + pb - dh * (kh - 1) - 1) // sh + 1
    ow = (wd + pl + pr - dw * (kw - 1) - 1) // sw + 1
    out = np.empty((n, o, oh, ow), dtype=np.int32)
    x = np.ascontiguousarray(x)
    w = np.ascontiguousarray(w)
    zwv = None
    zw_arr = np.asarray(zw)
    if zw_arr.ndim != 0:
        zwv = np.ascontiguousarray(zw_arr.astype(np.int32))
    rc = lib.oracle_qnn_conv2d(x.ctypes.data, int(x.dtype == np.uint8), w.ctypes.data, int(w.dtype == np.uint8),
                               out.ctypes.data, n, c, h, wd, o, kh, kw, sh, sw, pt, pl, pb, pr, dh, dw,
                               int(a["groups"]), int(za), int(zw_arr) if zwv is None else 0,
                               None if zwv is None else zwv.ctypes.data, threads)
    assert rc == 0
    return out


def _dense_c(x, w, za, zw, threads):
    from . import c_lib
    lib = c_lib()
    m, k = x.shape
    nn_ = w.shape[0]
    out = np.empty((m, nn_), dtype=np.int32)
    x = np.ascontiguousarray(x)
    w = np.ascontiguousarray(w)
    zw_arr = np.asarray(zw)
    zwv = None if zw_arr.ndim == 0 else np.ascontiguousarray(zw_arr.astype(np.int32))
    rc = lib.oracle_qnn_dense(x.ctypes.data, int(x.dtype == np.uint8), w.ctypes.data, int(w.dtype == np.uint8),
                              out.ctypes.data, m, k, nn_, int(za), int(zw_arr) if zwv is None else 0,
                              None if zwv is None else zwv.ctypes.data, threads)
    assert rc == 0
    return out


def _resolve_rounding(attrs):
    r = attrs.get("rounding", "None")
    if r in (None, "None"):
        r = attrs.get("cfg_rounding") or "UPWARD"
    return r


def _resolve_compute_dtype(attrs):
    """SelectRequntizeParameter for compute_dtype (qnn/utils.cc:231-245): the op's own attribute,
    else the requantize_config in effect, else int64 (llvm without -mcpu, requantize_config.h:53-72)."""
    cd = attrs.get("compute_dtype", "None")
    if cd in (None, "None"):
        cd = attrs.get("cfg_compute_dtype") or "int64"
    return cd


def eval_call(call, args, backend: str = "numpy", threads: int = 1):
    op = call.op
    a = call.attrs
    from . import realize_ref  # realized relay.quantize graphs and their float ops
    out = realize_ref.eval_call(call, args)
    if out is not None:
        return out
    if op == "qnn.conv2d":
        x, w = args[0], args[1]
        za, zw = _const(call.args[2]), _const(call.args[3])
        # NHWC data / HWIO, OHWI, HWOI kernels: the same contraction on the transposed operands, the
        # result in the data layout (Conv2DRel: out_layout defaults to data_layout)
        dl, kl = a.get("data_layout", "NCHW"), a.get("kernel_layout", "OIHW")
        if dl == "NHWC":
            x = np.ascontiguousarray(x.transpose(0, 3, 1, 2))
        if kl != "OIHW":
            w = np.ascontiguousarray(w.transpose([kl.index(ch) for ch in "OIHW"]))
        mult = a.get("depthwise_multiplier", 1)
        if mult > 1:
            # Conv2DRel's depthwise weight (C, M, KH, KW): output channel c * M + m reads [c, m]
            # (src/relay/op/nn/convolution.cc:243-274; topi depthwise_conv2d_nchw)
            w = w.reshape(w.shape[0] * w.shape[1], 1, w.shape[2], w.shape[3])
            if np.ndim(zw):
                zw = np.repeat(np.asarray(zw).reshape(-1), mult)
        if backend == "c":
            out = _conv_c(x, w, za, zw, a, threads)
        else:
            out = ref.qnn_conv2d(x, w, za, zw, strides=a["strides"], padding=a["padding"], dilation=a["dilation"],
                                 groups=a["groups"])
        return np.ascontiguousarray(out.transpose(0, 2, 3, 1)) if dl == "NHWC" else out
    if op == "qnn.dense":
        x, w = args[0], args[1]
        za, zw = _const(call.args[2]), _const(call.args[3])
        if backend == "c":
            return _dense_c(x, w, za, zw, threads)
        return ref.qnn_dense(x, w, za, zw)
    if op == "qnn.requantize":
        return ref.requantize(args[0], _const(call.args[1]), _const(call.args[2]), _const(call.args[3]),
                              _const(call.args[4]), axis=a["axis"], rounding=_resolve_rounding(a),
                              out_dtype=a["out_dtype"], compute_dtype=_resolve_compute_dtype(a))
    if op in ("qnn.add", "qnn.subtract", "qnn.mul"):
        c = [_const(call.args[i]) for i in range(2, 8)]
        fn = {"qnn.add": ref.qnn_add, "qnn.subtract": ref.qnn_subtract, "qnn.mul": ref.qnn_mul}[op]
        # every inner Requantize takes the requantize_config's rounding (qnn/utils.h:106-122)
        return fn(args[0], args[1], *c, lhs_axis=a.get("lhs_axis", -1), rhs_axis=a.get("rhs_axis", -1),
                  rounding=_resolve_rounding(a), compute_dtype=_resolve_compute_dtype(a))
    if op in ("qnn.concatenate", "qnn.leaky_relu") and _resolve_compute_dtype(a) != "int64":
        raise NotImplementedError(f"{op} under compute_dtype={_resolve_compute_dtype(a)}: not restated")
    if op == "qnn.concatenate":
        scales = [_const(f) for f in call.args[1].fields]
        zps = [_const(f) for f in call.args[2].fields]
        return ref.qnn_concatenate(args[0], scales, zps, _const(call.args[3]), _const(call.args[4]), axis=a["axis"],
                                   rounding=_resolve_rounding(a))
    if op == "qnn.leaky_relu":
        return ref.qnn_leaky_relu(args[0], a["alpha"], *[_const(call.args[i]) for i in range(1, 5)],
                                  rounding=_resolve_rounding(a))
    if op in ref.unary_functions():
        return ref.qnn_unary(op, args[0], *[_const(call.args[i]) for i in range(1, 5)])
    if op == "qnn.batch_matmul":
        return ref.qnn_batch_matmul(args[0], args[1], _const(call.args[2]), _const(call.args[3]))
    if op == "qnn.conv2d_transpose":
        x, w = args[0], args[1]
        dl, kl = a.get("data_layout", "NCHW"), a.get("kernel_layout", "IOHW")
        if dl == "NHWC":
            x = np.ascontiguousarray(x.transpose(0, 3, 1, 2))
        if kl != "IOHW":
            w = np.ascontiguousarray(w.transpose([kl.index(ch) for ch in "IOHW"]))
        za = np.asarray(_const(call.args[2])).reshape(-1)[0]
        zw = np.asarray(_const(call.args[3]))
        out = ref.qnn_conv2d_transpose(x, w, za, zw if zw.size > 1 else zw.reshape(-1)[0], strides=a["strides"],
                                       padding=a["padding"], output_padding=a["output_padding"], groups=a["groups"])
        return np.ascontiguousarray(out.transpose(0, 2, 3, 1)) if dl == "NHWC" else out
    if op == "qnn.quantize":
        return ref.quantize(args[0], _const(call.args[1]), _const(call.args[2]), axis=a["axis"],
                            out_dtype=a["out_dtype"])
    if op == "qnn.dequantize":
        return ref.dequantize(args[0], _const(call.args[1]), _const(call.args[2]), axis=a["axis"])
    if op == "qnn.simulated_quantize":
        return ref.simulated_quantize(args[0], int(np.asarray(args[1]).reshape(-1)[0]), args[2], args[3],
                                      axis=a.get("axis", -1))
    if op == "qnn.simulated_dequantize":
        return ref.simulated_dequantize(args[0], int(np.asarray(args[1]).reshape(-1)[0]), args[2], args[3],
                                        axis=a.get("axis", -1))
    if op == "transpose":
        return np.ascontiguousarray(np.transpose(args[0], a["axes"]))
    if op == "nn.bias_add":
        return ref.bias_add(args[0], args[1], axis=a["axis"])
    if op in ("tachikoma.qnn.conv2d", "tachikoma.qnn.dense"):
        from . import tachikoma_ref
        if op == "tachikoma.qnn.conv2d":
            acc = ref.qnn_conv2d(args[0], args[1], 0, 0, strides=a["strides"], padding=a["padding"],
                                 dilation=a["dilation"], groups=a["groups"])
        else:
            acc = ref.qnn_dense(args[0], args[1], 0, 0)
        po = a["postops"]
        return tachikoma_ref.postops(acc, po, call.dtype, sum_src=args[2] if len(args) > 2 else None,
                                     channel_axis=1, clip=po["clip"])
    if op == "clip":
        return ref.clip(args[0], a["a_min"], a["a_max"])
    if op == "nn.relu":
        return ref.relu(args[0])
    if op == "cast":
        return ref.cast(args[0], a["dtype"])
    if op == "nn.max_pool2d":
        return ref.max_pool2d(args[0], a["pool_size"], a["strides"], a["padding"], a["dilation"])
    if op == "nn.avg_pool2d":
        return ref.avg_pool2d(args[0], a["pool_size"], a["strides"], a["padding"], a["dilation"],
                              a.get("count_include_pad", False))
    if op == "nn.global_avg_pool2d":
        return ref.global_avg_pool2d(args[0])
    if op == "nn.batch_flatten":
        return ref.batch_flatten(args[0])
    if op == "reshape":
        return ref.reshape(args[0], a["newshape"])
    if op == "nn.pad":
        return ref.pad(args[0], a["pad_width"], args[1])
    raise NotImplementedError(op)


def calibrate(mod, params: Dict[str, np.ndarray], inputs: Dict[str, np.ndarray], backend: str = "numpy",
              threads: Optional[int] = None, keep=None) -> Dict[str, np.ndarray]:
    """Trace.calibrate: returns {symbol name: output} for every input and op (params excluded).

    ``keep``: optional callable(name, array) -> bool deciding whether a record is kept after
    its consumers no longer need it (memory bound for big models); default keeps all."""
    func = mod["main"] if hasattr(mod, "functions") else mod
    body = func.body if hasattr(func, "body") else func
    nodes = _post_order(body)
    if threads is None:
        threads = len(os.sched_getaffinity(0))
    values: Dict[int, np.ndarray] = {}
    records: Dict[str, np.ndarray] = {}
    counter = 0
    # last use of each node, to drop intermediates when keep() says so
    last_use = {}
    for i, node in enumerate(nodes):
        for a in getattr(node, "args", []):
            last_use[id(a)] = i
    for i, node in enumerate(nodes):
        kind = type(node).__name__
        if kind == "Var":
            if node.name_hint in params:
                values[id(node)] = np.asarray(params[node.name_hint])
            else:
                v = np.asarray(inputs[node.name_hint])
                values[id(node)] = v
                records[node.name_hint] = v
        elif kind == "Constant":
            values[id(node)] = node.data
        elif kind == "Tuple":
            # a tuple is no op: it has no record and takes no symbol name (MRT's expr2symbol
            # names Calls and TupleGetItems, python/tvm/mrt/symbol.py:212-253)
            values[id(node)] = [values[id(f)] for f in node.fields]
        elif kind == "Call" and node.op == "reshape" and type(node.args[0]).__name__ == "Constant":
            # reshape of a constant (the [-1] reshapes the simulated_(de)quantize constructors put
            # around their scale / zero point, relay/qnn/op/qnn.py:253-255): FoldConstant folds it
            # into a constant when the reference builds the graph, so it is no op and no record
            values[id(node)] = np.reshape(node.args[0].data, node.shape)
        elif kind == "Call":
            name = f"%{counter}"
            counter += 1
            args = [values[id(a)] for a in node.args]
            out = eval_call(node, args, backend, threads)
            # the batch axis may be a subset of the graph's (samples are independent)
            assert tuple(out.shape[1:]) == tuple(node.shape[1:]) or tuple(out.shape) == tuple(node.shape), \
                (name, node.op, out.shape, node.shape)
            assert str(out.dtype) == node.dtype, (name, node.op, out.dtype, node.dtype)
            values[id(node)] = out
            if keep is None or keep(name, out):
                records[name] = out
        for a in getattr(node, "args", []):
            if last_use.get(id(a)) == i and type(a).__name__ == "Call" and id(a) != id(body):
                values.pop(id(a), None)
    return records

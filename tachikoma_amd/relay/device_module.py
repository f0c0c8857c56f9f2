"""Device-side module: HBM buffers + the native node list (tk_module).

Memory layout in HBM (one GPU, one batch shard):
  * params: uploaded once; MFMA convs additionally hold a packed
    [Cout_pad][KH][KW][Cin_pad] int8 copy and int32 per-channel weight sums;
  * graph inputs and EVERY op output get their own buffer (no storage-pool
    reuse as in graph_executor.cc:356-464), so each output stays addressable
    for the trace copy-out until the step ends — ResNet-50 at 64 samples is
    ~7 GB, nothing next to 288 GB;
  * every tensor read by an MFMA conv has an int8 "shadow", channel-blocked
    [C_pad16/16][N·H·W][16]: written directly by the producing fused conv block's epilogue, or by
    a shadow node right before the first conv that reads it.

Nodes: one per ExecGroup (build_module.exec_groups) — a fused conv/dense layer
block or residual (qnn.add → clip) block writes all of its ops' outputs (each a
separate trace record) from one kernel.
"""
from __future__ import annotations

import atexit
import ctypes
import sys
import weakref
from typing import Callable, Dict, List, Optional

import numpy as np

from .. import _lib
from .build_module import ExecGroup, Plan, PlanOp, exec_groups
from .qnn import legalize as _legalize
from .qnn import op as _qnn


def _torch():
    import torch
    return torch


def torch_dtype(name: str):
    torch = _torch()
    return {"int8": torch.int8, "uint8": torch.uint8, "int16": torch.int16, "int32": torch.int32,
            "int64": torch.int64, "float32": torch.float32}[name]


# Every DeviceModule whose native module is alive.  The atexit hook closes them before the
# interpreter finalises (atexit runs first, LIFO after torch's own hooks were registered at import),
# so no tk_module_destroy -- HIP graph / event / stream / hipFree calls -- ever runs from a finaliser
# or after the HIP runtime's static destructors (the round-4 exit SIGSEGV under rocprofv3 was raised
# inside __cxa_finalize).
_LIVE: "weakref.WeakSet[DeviceModule]" = weakref.WeakSet()


@atexit.register
def close_all() -> None:
    """Close every live DeviceModule (also callable directly, e.g. before os._exit)."""
    for m in list(_LIVE):
        try:
            m.close()
        except Exception as e:  # report, keep closing the others
            sys.stderr.write(f"[tachikoma] closing a module at exit failed: {e}\n")


def tune_table_digest(entries) -> str:
    """Digest of a find-step choice: sorted (records, algo) pairs (entries of ``tuning`` or of a
    tune table)."""
    import hashlib
    import json
    return hashlib.sha256(json.dumps(sorted((list(e["records"]), int(e["algo"])) for e in entries)).encode()
                          ).hexdigest()[:16]


class DeviceModule:
    def __init__(self, plan: Plan, params: Dict[str, np.ndarray], dev=None, fuse: bool = True, tune=True):
        """``tune``: True runs the find step (tk_module_tune) on this GPU, False keeps the library's
        own kernel choice, a tune table (``tuning_table()`` output, or the path of its JSON file)
        replays a saved find step so that a profile and a timed run use the same kernels."""
        torch = _torch()
        if not torch.cuda.is_available():
            raise _lib.TachikomaError("no MI355X visible: the engine runs on the GPU only (no CPU fallback)")
        self.lib = _lib.load()
        self.plan = plan
        self.device = torch.device("cuda", 0) if dev is None else _as_torch_device(dev)
        self.buffers: Dict[str, "torch.Tensor"] = {}
        self._keep: List[object] = []
        self.node_records: List[List[str]] = []  # tk node index -> record names of its outputs
        self.node_kinds: List[str] = []
        self.node_native_kinds: List[int] = []  # tk_node kind (TK_NODE_*) of each node
        # param name -> re-derivations of the build-time buffers computed from it (packed MFMA
        # weights + weight sums), re-run whenever the param's device copy is rewritten
        self._derived: Dict[str, List[Callable[[int], None]]] = {}
        self.groups = exec_groups(plan, fuse=fuse)
        self.tuning: List[dict] = []
        self.tables: Dict[str, object] = {}  # qnn unary ops: op name -> its device lookup table
        # runs as one replayed HIP graph (tk_module_run_graph) instead of host-issued nodes and
        # copies; GraphModule.pick_run_mode chooses by timing both on this host
        self.use_graph = False
        with torch.cuda.device(self.device):
            self._alloc(params)
            self._build_nodes()
            if isinstance(tune, (str, dict)):
                self.apply_tuning(tune)
            elif tune:
                self.tune()

    # ------------------------------------------------------------ setup
    def _alloc(self, params):
        torch = _torch()
        for t in self.plan.inputs:
            self.buffers[t.name] = torch.zeros(t.shape, dtype=torch_dtype(t.dtype), device=self.device)
        for t in self.plan.params:
            self.buffers[t.name] = torch.from_numpy(np.ascontiguousarray(params[t.name])).to(self.device)
        for op in self.plan.ops:
            self.buffers[op.name] = torch.empty(op.out.shape, dtype=torch_dtype(op.out.dtype), device=self.device)
        self._alloc_layouts()

    # NHWC data / HWIO, OHWI, HWOI kernels of qnn.conv2d (convolution.cc:718-722): the NCHW / OIHW
    # kernels run between device transposes into untraced buffers named "<op>:nchw_in",
    # "<op>:oihw_w" (re-derived from the param whenever it is rewritten) and "<op>:nchw_out"; the
    # record itself stays in the op's own layout.
    _TO_NCHW = (0, 3, 1, 2)
    _TO_NHWC = (0, 2, 3, 1)

    def _alloc_layouts(self):
        torch = _torch()
        self.layout: Dict[str, Dict[str, object]] = {}
        for op in self.plan.ops:
            if op.op == "qnn.conv2d_transpose":
                self._alloc_transpose_layout(op)
                continue
            if op.op != "qnn.conv2d":
                continue
            dl, kl = op.attrs.get("data_layout", "NCHW"), op.attrs.get("kernel_layout", "OIHW")
            mult = op.attrs.get("depthwise_multiplier", 1)
            if dl == "NCHW" and kl == "OIHW" and mult == 1:
                continue
            wt = self.plan.tensor(op.inputs[1])
            ws = tuple(wt.shape[kl.index(ch)] for ch in "OIHW")
            # the grouped-conv weight the kernels read: a depthwise-multiplier weight (C, M, KH, KW)
            # is the same bytes as (C * M, 1, KH, KW) (out channel c * M + m reads [c, m])
            w_shape = (ws[0] * ws[1], 1, ws[2], ws[3]) if mult > 1 else ws
            L: Dict[str, object] = {"x": op.inputs[0], "w": op.inputs[1], "y": op.name, "w_shape": w_shape}
            if dl == "NHWC":
                xt = self.plan.tensor(op.inputs[0])
                n_, h_, w_, c_ = xt.shape
                L["x"] = f"{op.name}:nchw_in"
                self.buffers[L["x"]] = torch.empty((n_, c_, h_, w_), dtype=torch_dtype(xt.dtype), device=self.device)
                n_, oh, ow, o_ = op.out.shape
                L["y"] = f"{op.name}:nchw_out"
                self.buffers[L["y"]] = torch.empty((n_, o_, oh, ow), dtype=torch.int32, device=self.device)
            if kl != "OIHW":
                perm = tuple(kl.index(ch) for ch in "OIHW")
                L["w"] = f"{op.name}:oihw_w"
                self.buffers[L["w"]] = torch.empty(tuple(wt.shape[k] for k in perm), dtype=torch_dtype(wt.dtype),
                                                   device=self.device)
                self._register_transpose(op.inputs[1], L["w"], perm)
            self.layout[op.name] = L

    def _alloc_transpose_layout(self, op: PlanOp) -> None:
        """qnn.conv2d_transpose runs on NCHW data and an IOHW weight: NHWC data goes through
        "<op>:nchw_in" / "<op>:nchw_out" and any other kernel layout through "<op>:iohw_w"."""
        torch = _torch()
        dl, kl = op.attrs["data_layout"], op.attrs["kernel_layout"]
        L: Dict[str, object] = {"x": op.inputs[0], "w": op.inputs[1], "y": op.name}
        if dl == "NHWC":
            xt = self.plan.tensor(op.inputs[0])
            n_, h_, w_, c_ = xt.shape
            L["x"] = f"{op.name}:nchw_in"
            self.buffers[L["x"]] = torch.empty((n_, c_, h_, w_), dtype=torch_dtype(xt.dtype), device=self.device)
            n_, oh, ow, o_ = op.out.shape
            L["y"] = f"{op.name}:nchw_out"
            self.buffers[L["y"]] = torch.empty((n_, o_, oh, ow), dtype=torch.int32, device=self.device)
        if kl != "IOHW":
            wt = self.plan.tensor(op.inputs[1])
            perm = tuple(kl.index(ch) for ch in "IOHW")
            L["w"] = f"{op.name}:iohw_w"
            self.buffers[L["w"]] = torch.empty(tuple(wt.shape[k] for k in perm), dtype=torch_dtype(wt.dtype),
                                               device=self.device)
            self._register_transpose(op.inputs[1], L["w"], perm)
        if dl != "NCHW" or kl != "IOHW":
            self.layout[op.name] = L

    def _transpose_attrs(self, perm):
        ta = _lib.tk_transpose_attrs()
        ta.ndim = len(perm)
        for k, p in enumerate(perm):
            ta.perm[k] = p
        return ta

    def _register_transpose(self, src: str, dst: str, perm) -> None:
        """dst = transpose(src) now, and again whenever the param ``src`` is rewritten."""
        x, y = self._ref(src), self._ref(dst)
        ta = self._transpose_attrs(perm)
        self._keep.append(ta)

        def run(s: int) -> None:
            _lib.check(self.lib.tk_transpose(x.ptr, y.ptr, ctypes.byref(ta), ctypes.c_void_p(s)), f"transpose {src}")
        run(_lib.stream_handle())
        self._derived.setdefault(src, []).append(run)

    def _conv_io(self, op: PlanOp):
        """(data buffer, weight buffer) the NCHW / OIHW conv kernels read for ``op``."""
        L = self.layout.get(op.name)
        return (L["x"], L["w"]) if L else (op.inputs[0], op.inputs[1])

    def _conv_refs(self, op: PlanOp):
        """TensorRefs of the NCHW data and the OIHW grouped-conv weight for ``op``."""
        xn, wn = self._conv_io(op)
        L = self.layout.get(op.name)
        return self._ref(xn), (self._view_ref(wn, L["w_shape"]) if L else self._ref(wn))

    def _ref(self, name: str) -> _lib.TensorRef:
        r = _lib.TensorRef.from_torch(self.buffers[name])
        self._keep.append(r)
        return r

    def _dev_const(self, arr: np.ndarray):
        """A node constant on the device in its own dtype (kept alive with the module)."""
        t = _torch().from_numpy(np.ascontiguousarray(arr)).to(self.device)
        self._keep.append(t)
        return t

    def _dev_i32(self, arr: np.ndarray):
        torch = _torch()
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int32)).to(self.device)
        self._keep.append(t)
        return t

    def _scratch(self, nbytes: int, zero: bool = False):
        torch = _torch()
        alloc = torch.zeros if zero else torch.empty
        t = alloc(max(int(nbytes), 16), dtype=torch.uint8, device=self.device)
        self._keep.append(t)
        return t

    def _conv_attrs(self, ca, op: PlanOp):
        a = op.attrs
        ca.strides[:] = list(a["strides"])
        ca.padding[:] = list(a["padding"])
        ca.dilation[:] = list(a["dilation"])
        ca.groups = a["groups"]
        ca.input_zero_point = a["input_zero_point"]
        ca.kernel_zero_point = a["kernel_zero_point"]
        if "kernel_zero_points" in op.consts:
            ca.kernel_zero_points = self._dev_i32(op.consts["kernel_zero_points"]).data_ptr()

    def _dense_attrs(self, da, op: PlanOp):
        a = op.attrs
        da.input_zero_point = a["input_zero_point"]
        da.kernel_zero_point = a["kernel_zero_point"]
        if "kernel_zero_points" in op.consts:
            da.kernel_zero_points = self._dev_i32(op.consts["kernel_zero_points"]).data_ptr()

    def _fill_rq(self, r, op: PlanOp):
        a = op.attrs
        r.mode = a["mode"]
        r.axis = a["channel_axis"]
        r.multiplier = a.get("multiplier", 0)
        r.shift = a.get("shift", 0)
        if "multipliers" in op.consts:
            r.multipliers = self._dev_i32(op.consts["multipliers"]).data_ptr()
            r.shifts = self._dev_i32(op.consts["shifts"]).data_ptr()
        r.input_zero_point = a["input_zero_point"]
        if "input_zero_points" in op.consts:
            r.input_zero_points = self._dev_i32(op.consts["input_zero_points"]).data_ptr()
        r.output_zero_point = a["output_zero_point"]

    def _fp_side(self, r, a, consts, prefix: str, axis: int, zp_key: str, zps_key: str, zp_out: int) -> None:
        """One tk_requantize_fp_attrs from a lowered plan's ``{prefix}fp_*`` attrs / consts."""
        r.bits = a[f"{prefix}fp_bits"]
        r.rounding = _lib.TK_ROUND_UPWARD if a["rounding"] == "UPWARD" else _lib.TK_ROUND_TONEAREST
        r.axis = axis
        r.scaled = a[f"{prefix}fp_scaled"]
        r.multiplier = a[f"{prefix}fp_multiplier"]
        if f"{prefix}fp_multipliers" in consts:
            r.multipliers = self._dev_const(np.asarray(consts[f"{prefix}fp_multipliers"], np.float64)).data_ptr()
        r.input_zero_point = a[zp_key]
        if zps_key in consts:
            r.input_zero_points = self._dev_i32(consts[zps_key]).data_ptr()
        r.output_zero_point = zp_out

    def _fill_rq_fp(self, r, op: PlanOp):
        """tk_requantize_fp_attrs of a qnn.requantize built under a float compute_dtype."""
        a = op.attrs
        self._fp_side(r, a, op.consts, "", a["channel_axis"], "input_zero_point", "input_zero_points",
                      a["output_zero_point"])

    def _fill_binary_fp(self, qb, op: PlanOp) -> None:
        """tk_qnn_binary_fp_attrs from a lowered qnn.add / subtract / mul (float compute_dtype)."""
        a = op.attrs
        qb.op = _lib.TK_QB[op.op]
        mul = op.op == "qnn.mul"
        for side in ("lhs", "rhs", "out"):
            if f"{side}_mode" not in a:
                continue
            r = getattr(qb, side)
            if f"{side}_fp_bits" in a:
                self._fp_side(r, a, op.consts, f"{side}_", a[f"{side}_axis"], f"{side}_zero_point", f"{side}_zero_points",
                              0 if mul and side != "out" else a["output_zero_point"])
            else:  # an upcast side (add / subtract) or a mul operand: only its zero point(s) are read
                r.bits = 32 if a["compute_dtype"] == "float32" else 64
                r.axis = a[f"{side}_axis"]
                r.input_zero_point = a[f"{side}_zero_point"]
                if f"{side}_zero_points" in op.consts:
                    r.input_zero_points = self._dev_i32(op.consts[f"{side}_zero_points"]).data_ptr()
        qb.lhs_upcast = a.get("lhs_upcast", 0)
        qb.rhs_upcast = a.get("rhs_upcast", 0)
        qb.output_zero_point = a["output_zero_point"]

    def _is_mfma_conv(self, op: PlanOp) -> bool:
        ca = _lib.tk_conv2d_attrs()
        self._conv_attrs(ca, op)
        x, w = self._conv_refs(op)
        ws = self.lib.tk_qnn_conv2d_workspace_bytes(x.ptr, w.ptr, ctypes.byref(ca))
        if ws < 0:
            _lib.check(-3, f"{op.name} qnn.conv2d workspace")
        return ws > 0

    def _build_nodes(self):
        torch = _torch()
        stream = _lib.stream_handle()
        nodes: List[_lib.tk_node] = []
        # tensors read by MFMA convs need a shadow
        conv_ops = [g.ops[0] for g in self.groups if g.ops[0].op in ("qnn.conv2d", "tachikoma.qnn.conv2d")]
        mfma = {op.name: self._is_mfma_conv(op) for op in conv_ops}
        shadow_bufs: Dict[str, object] = {}
        # 8-bit max pools read their input's shadow too (16 channels per load) and write
        # their own output's shadow when an MFMA conv reads it
        pool_ops = [g.ops[0] for g in self.groups if g.ops[0].op == "nn.max_pool2d" and
                    g.ops[0].out.dtype in ("int8", "uint8") and len(g.ops[0].out.shape) == 4]
        need = [self._conv_io(op)[0] for op in conv_ops if mfma[op.name]] + [op.inputs[0] for op in pool_ops]
        for name in need:
            if name not in shadow_bufs:
                x = self._ref(name)
                shadow_bufs[name] = self._scratch(self.lib.tk_conv2d_shadow_bytes(x.ptr), zero=True)
        pool_names = {op.name for op in pool_ops}
        shadow_ready = set()

        def emit(n, kind, records):
            nodes.append(n)
            self.node_kinds.append(kind)
            self.node_native_kinds.append(int(n.kind))
            self.node_records.append(records)

        def ensure_shadow(name: str):
            if name in shadow_ready:
                return
            sn = _lib.tk_node()
            sn.kind = _lib.NODE_KINDS["shadow"]
            sn.n_inputs = 1
            sn.inputs[0] = self._ref(name).ptr
            sn.n_outputs = 0
            sn.ext[0] = shadow_bufs[name].data_ptr()
            emit(sn, "shadow", [])
            shadow_ready.add(name)

        for g in self.groups:
            head = g.ops[0]
            n = _lib.tk_node()
            if g.kind in ("tachikoma.qnn.conv2d", "tachikoma.qnn.dense"):
                self._emit_composite(head, mfma, shadow_bufs, ensure_shadow, stream, emit)
                continue
            if g.kind in ("conv_block", "dense_block"):
                bias_op, rq_op = g.ops[1], g.ops[2]
                ins = [self._ref(head.inputs[0]), self._ref(head.inputs[1]), self._ref(bias_op.inputs[1])]
                outs = [self._ref(o.name) for o in g.ops]
                ba = n.attrs.block
                self._fill_rq(ba.requantize, rq_op)
                add = g.add
                if add is not None:
                    # residual join: the block's requantize output is one qnn.add operand
                    ba.has_add = 1
                    ba.block_is_rhs = int(add.inputs[1] == rq_op.name)
                    residual = add.inputs[0] if ba.block_is_rhs else add.inputs[1]
                    ins.append(self._ref(residual))
                    _fill_qnn_add(ba.add, add.attrs)
                if g.last.op in ("clip", "nn.relu"):
                    ba.has_clip = 1
                    ba.clip_min, ba.clip_max = g.last.attrs["lo"], g.last.attrs["hi"]
                if g.kind == "conv_block":
                    n.kind = _lib.NODE_KINDS["conv_block"]
                    self._conv_attrs(ba.conv, head)
                    self._prep_conv(n, head, ins, mfma[head.name], shadow_bufs, ensure_shadow, stream)
                    if g.last.name in shadow_bufs:
                        # the epilogue writes the shadow the next MFMA conv reads
                        n.ext[4] = shadow_bufs[g.last.name].data_ptr()
                        shadow_ready.add(g.last.name)
                elif self._dense_as_conv(n, g, head, ins, outs, emit, stream):
                    pass
                else:
                    n.kind = _lib.NODE_KINDS["dense_block"]
                    self._dense_attrs(ba.dense, head)
                    n.ext[0] = self._scratch(self.lib.tk_qnn_dense_workspace_bytes(ins[0].ptr, ins[1].ptr)).data_ptr()
            elif g.kind == "add_block":
                n.kind = _lib.NODE_KINDS["add_block"]
                ins = [self._ref(x) for x in head.inputs[:2]]
                outs = [self._ref(o.name) for o in g.ops]
                ab = n.attrs.add_block
                _fill_qnn_add(ab.add, head.attrs)
                if len(g.ops) == 2:
                    ab.has_clip = 1
                    ab.clip_min, ab.clip_max = g.ops[1].attrs["lo"], g.ops[1].attrs["hi"]
                if g.last.name in shadow_bufs and len(head.out.shape) == 4:
                    n.ext[4] = shadow_bufs[g.last.name].data_ptr()
                    shadow_ready.add(g.last.name)
            else:
                op = head
                kind = op.op
                ins = [self._ref(x) for x in op.inputs]
                outs = [self._ref(op.name)]
                a = op.attrs
                if kind == "qnn.conv2d" and op.name in self.layout:
                    self._emit_layout_conv(n, op, mfma[op.name], shadow_bufs, ensure_shadow, stream, emit)
                    continue
                if kind == "qnn.conv2d_transpose":
                    self._emit_conv2d_transpose(n, op, emit)
                    continue
                if kind == "qnn.conv2d":
                    n.kind = _lib.NODE_KINDS["qnn.conv2d"]
                    self._conv_attrs(n.attrs.conv2d, op)
                    self._prep_conv(n, op, ins, mfma[op.name], shadow_bufs, ensure_shadow, stream)
                elif kind == "qnn.dense":
                    n.kind = _lib.NODE_KINDS["qnn.dense"]
                    self._dense_attrs(n.attrs.dense, op)
                    n.ext[0] = self._scratch(self.lib.tk_qnn_dense_workspace_bytes(ins[0].ptr, ins[1].ptr)).data_ptr()
                elif kind == "qnn.requantize" and a.get("compute_dtype", "int64") != "int64":
                    n.kind = _lib.NODE_KINDS["requantize_fp"]
                    self._fill_rq_fp(n.attrs.requantize_fp, op)
                elif kind == "qnn.requantize":
                    n.kind = _lib.NODE_KINDS["qnn.requantize"]
                    self._fill_rq(n.attrs.requantize, op)
                elif kind in ("qnn.add", "qnn.subtract", "qnn.mul") and a.get("compute_dtype", "int64") != "int64":
                    n.kind = _lib.NODE_KINDS["qnn_binary_fp"]
                    self._fill_binary_fp(n.attrs.qnn_binary_fp, op)
                elif kind == "qnn.add" and a.get("per_tensor"):
                    n.kind = _lib.NODE_KINDS["qnn.add"]
                    _fill_qnn_add(n.attrs.qnn_add, a)
                elif kind in ("qnn.add", "qnn.subtract", "qnn.mul"):
                    n.kind = _lib.NODE_KINDS["qnn_binary"]
                    self._fill_binary(n.attrs.qnn_binary, op)
                elif kind in ("qnn.quantize", "qnn.dequantize"):
                    n.kind = _lib.NODE_KINDS[kind]
                    qa = n.attrs.qparams
                    qa.axis = a["axis"]
                    qa.scale = a["scale"]
                    qa.zero_point = a["zero_point"]
                    if "scales" in op.consts:
                        t = _torch().from_numpy(np.ascontiguousarray(op.consts["scales"], np.float32)).to(self.device)
                        self._keep.append(t)
                        qa.scales = t.data_ptr()
                    if "zero_points" in op.consts:
                        qa.zero_points = self._dev_i32(op.consts["zero_points"]).data_ptr()
                elif kind == "qnn.concatenate":
                    n.kind = _lib.NODE_KINDS[kind]
                    ca = n.attrs.concat
                    ca.axis = a["axis"]
                    ca.n = len(ins)
                    for k, pl in enumerate(a["inputs"]):
                        ca.requant[k] = pl["requant"]
                        r = ca.rq[k]
                        r.mode, r.axis = pl["mode"], -1
                        r.multiplier, r.shift = pl["multiplier"], pl["shift"]
                        r.input_zero_point, r.output_zero_point = pl["input_zero_point"], pl["output_zero_point"]
                elif kind == "transpose":
                    n.kind = _lib.NODE_KINDS["transpose"]
                    n.attrs.transpose = self._transpose_attrs(a["axes"])
                elif kind == "qnn.leaky_relu":
                    n.kind = _lib.NODE_KINDS[kind]
                    la = n.attrs.leaky_relu
                    r = la.rq
                    r.mode, r.axis, r.multiplier, r.shift = a["mode"], -1, a["multiplier"], a["shift"]
                    r.input_zero_point, r.output_zero_point = a["input_zero_point"], a["output_zero_point"]
                    la.upcast = a["upcast"]
                    la.input_zero_point, la.output_zero_point = a["input_zero_point"], a["output_zero_point"]
                    la.alpha_multiplier, la.alpha_shift = a["alpha_multiplier"], a["alpha_shift"]
                    la.zp_multiplier, la.zp_shift = a["zp_multiplier"], a["zp_shift"]
                elif kind in _qnn.UNARY_OPS:
                    n.kind = _lib.NODE_KINDS["lookup"]
                    table = _legalize.build_table(self.lib, kind, op.out.dtype, a["in_scale"], a["in_zero_point"],
                                                  a["out_scale"], a["out_zero_point"], self.device, stream)
                    self._keep.append(table)
                    self.tables[op.name] = table
                    n.ext[0] = table.data_ptr()
                elif kind in ("qnn.simulated_quantize", "qnn.simulated_dequantize"):
                    n.kind = _lib.NODE_KINDS[kind]
                    sq = n.attrs.simq
                    sq.axis = a["axis"]
                    sq.n_scales, sq.n_zero_points = a["n_scales"], a["n_zero_points"]
                    # each parameter is a folded constant uploaded here or a graph tensor's buffer
                    # (read on the device when the node runs)
                    src = {key: (self._dev_const(op.consts[key]) if k < 0 else self.buffers[op.inputs[k]]).data_ptr()
                           for key, k in a["sources"].items()}
                    sq.dtype_code, sq.scales, sq.zero_points = src["dtype_code"], src["scales"], src["zero_points"]
                elif kind == "qnn.batch_matmul":
                    n.kind = _lib.NODE_KINDS[kind]
                    self._dense_attrs(n.attrs.dense, op)
                    ws = self.lib.tk_qnn_batch_matmul_workspace_bytes(ins[0].ptr, ins[1].ptr)
                    if ws < 0:
                        _lib.check(int(ws), f"{op.name} qnn.batch_matmul workspace")
                    n.ext[0] = self._scratch(ws).data_ptr()
                elif kind == "nn.bias_add":
                    n.kind = _lib.NODE_KINDS["nn.bias_add"]
                    n.attrs.bias_add.axis = a["axis"]
                elif kind in ("clip", "nn.relu"):
                    n.kind = _lib.NODE_KINDS["clip"]
                    n.attrs.clip.a_min = a["lo"]
                    n.attrs.clip.a_max = a["hi"]
                elif kind == "cast":
                    n.kind = _lib.NODE_KINDS["cast"]
                elif kind in ("nn.max_pool2d", "nn.avg_pool2d"):
                    n.kind = _lib.NODE_KINDS[kind]
                    if op.name in pool_names:
                        ensure_shadow(op.inputs[0])
                        n.ext[0] = shadow_bufs[op.inputs[0]].data_ptr()
                        if op.name in shadow_bufs:
                            n.ext[4] = shadow_bufs[op.name].data_ptr()
                            shadow_ready.add(op.name)
                    pa = n.attrs.pool2d
                    pa.pool_size[:] = list(a["pool_size"])
                    pa.strides[:] = list(a["strides"])
                    pa.padding[:] = list(a["padding"])
                    pa.dilation[:] = list(a["dilation"])
                    pa.count_include_pad = int(a.get("count_include_pad", False))
                elif kind == "nn.global_avg_pool2d":
                    n.kind = _lib.NODE_KINDS[kind]
                elif kind in ("nn.batch_flatten", "reshape", "annotation.stop_fusion", "annotation.cast_hint"):
                    n.kind = _lib.NODE_KINDS["copy"]
                elif kind == "nn.pad":
                    n.kind = _lib.NODE_KINDS["nn.pad"]
                    pa = n.attrs.pad
                    for d, (b_, a_) in enumerate(a["pad_width"]):
                        pa.before[d], pa.after[d] = b_, a_
                    if op.out.dtype == "float32":
                        pa.value_f = float(a["value"])
                    else:
                        pa.value_i = int(a["value"])
                elif kind == "ewise":
                    n.kind = _lib.NODE_KINDS["ewise"]
                    ew = n.attrs.ewise
                    ew.op = _lib.TK_EW[a["ew"]]
                    ew.rhs_kind = a["rhs_kind"]
                    ew.scalar_f = a.get("scalar_f", 0.0)
                    ew.scalar_i = a.get("scalar_i", 0)
                    ew.lo = a.get("lo", 0.0)
                    ew.hi = a.get("hi", 0.0)
                    ew.multiplier = a.get("multiplier", 0)
                    ew.shift = a.get("shift", 0)
                elif kind == "nn.conv2d":  # float32 (int8 ones are lowered to qnn.conv2d)
                    n.kind = _lib.NODE_KINDS["conv2d_f32"]
                    ca = n.attrs.conv2d
                    ca.strides[:] = list(a["strides"])
                    ca.padding[:] = list(a["padding"])
                    ca.dilation[:] = list(a["dilation"])
                    ca.groups = a["groups"]
                elif kind == "nn.dense":
                    n.kind = _lib.NODE_KINDS["dense_f32"]
                else:
                    raise _lib.TachikomaError(f"no device lowering for {kind}")
            n.n_inputs = len(ins)
            for k, r in enumerate(ins):
                n.inputs[k] = r.ptr
            n.n_outputs = len(outs)
            for k, r in enumerate(outs):
                n.outputs[k] = r.ptr
            emit(n, g.kind, [o.name for o in g.ops])
        torch.cuda.current_stream().synchronize()
        self._node_kind_codes = [int(n.kind) for n in nodes]
        self._nodes = nodes  # (their tensors and attrs describe a node's kernels: algo_info)
        arr = (_lib.tk_node * max(1, len(nodes)))(*nodes)
        handle = ctypes.c_void_p()
        _lib.check(self.lib.tk_module_create(arr, len(nodes), ctypes.byref(handle)), "tk_module_create")
        self.handle = handle
        _LIVE.add(self)
        self.n_nodes = len(nodes)

    def _fill_binary(self, qb, op: PlanOp) -> None:
        """tk_qnn_binary_attrs from a lowered qnn.add / qnn.subtract / qnn.mul."""
        a = op.attrs
        qb.op = _lib.TK_QB[op.op]
        for side in ("lhs", "rhs", "out"):
            if f"{side}_mode" not in a:
                continue
            r = getattr(qb, side)
            r.mode = a[f"{side}_mode"]
            r.axis = a[f"{side}_axis"]
            r.multiplier = a[f"{side}_multiplier"]
            r.shift = a[f"{side}_shift"]
            if f"{side}_multipliers" in op.consts:
                r.multipliers = self._dev_i32(op.consts[f"{side}_multipliers"]).data_ptr()
                r.shifts = self._dev_i32(op.consts[f"{side}_shifts"]).data_ptr()
            r.input_zero_point = a[f"{side}_zero_point"]
            if f"{side}_zero_points" in op.consts:
                r.input_zero_points = self._dev_i32(op.consts[f"{side}_zero_points"]).data_ptr()
            r.output_zero_point = a["output_zero_point"] if side != "lhs" or op.op != "qnn.mul" else 0
        if op.op == "qnn.mul":
            qb.lhs.output_zero_point = qb.rhs.output_zero_point = 0
        qb.lhs_upcast = a.get("lhs_upcast", 0)
        qb.rhs_upcast = a.get("rhs_upcast", 0)
        qb.output_zero_point = a["output_zero_point"]

    def _emit_layout_conv(self, n, op: PlanOp, is_mfma: bool, shadow_bufs, ensure_shadow, stream, emit) -> None:
        """qnn.conv2d with NHWC data and/or a non-OIHW kernel: [transpose data -> NCHW], the NCHW /
        OIHW conv into an int32 NCHW buffer, [transpose -> the NHWC record]."""
        L = self.layout[op.name]

        def transpose_node(src: str, dst: str, perm, records):
            t = _lib.tk_node()
            t.kind = _lib.NODE_KINDS["transpose"]
            t.attrs.transpose = self._transpose_attrs(perm)
            t.n_inputs, t.n_outputs = 1, 1
            t.inputs[0], t.outputs[0] = self._ref(src).ptr, self._ref(dst).ptr
            emit(t, "transpose", records)

        if L["x"] != op.inputs[0]:
            transpose_node(op.inputs[0], L["x"], self._TO_NCHW, [])
        ins = list(self._conv_refs(op))
        n.kind = _lib.NODE_KINDS["qnn.conv2d"]
        self._conv_attrs(n.attrs.conv2d, op)
        self._prep_conv(n, op, ins, is_mfma, shadow_bufs, ensure_shadow, stream)
        n.n_inputs, n.n_outputs = 2, 1
        n.inputs[0], n.inputs[1] = ins[0].ptr, ins[1].ptr
        n.outputs[0] = self._ref(L["y"]).ptr
        emit(n, "qnn.conv2d", [] if L["y"] != op.name else [op.name])
        if L["y"] != op.name:
            transpose_node(L["y"], op.name, self._TO_NHWC, [op.name])

    def _emit_conv2d_transpose(self, n, op: PlanOp, emit) -> None:
        """qnn.conv2d_transpose: [transpose NHWC data -> NCHW], the NCHW / IOHW kernel, [transpose ->
        the NHWC record]; a non-IOHW weight was transposed into "<op>:iohw_w" (re-derived on rewrite)."""
        L = self.layout.get(op.name, {"x": op.inputs[0], "w": op.inputs[1], "y": op.name})
        a = op.attrs

        def transpose_node(src: str, dst: str, perm, records):
            t = _lib.tk_node()
            t.kind = _lib.NODE_KINDS["transpose"]
            t.attrs.transpose = self._transpose_attrs(perm)
            t.n_inputs, t.n_outputs = 1, 1
            t.inputs[0], t.outputs[0] = self._ref(src).ptr, self._ref(dst).ptr
            emit(t, "transpose", records)

        if L["x"] != op.inputs[0]:
            transpose_node(op.inputs[0], L["x"], self._TO_NCHW, [])
        n.kind = _lib.NODE_KINDS["qnn.conv2d_transpose"]
        ta = n.attrs.conv2d_transpose
        ta.strides[:] = list(a["strides"])
        ta.padding[:] = list(a["padding"])
        ta.output_padding[:] = list(a["output_padding"])
        ta.groups = a["groups"]
        ta.input_zero_point = a["input_zero_point"]
        ta.kernel_zero_point = a["kernel_zero_point"]
        if "kernel_zero_points" in op.consts:
            ta.kernel_zero_points = self._dev_i32(op.consts["kernel_zero_points"]).data_ptr()
        n.n_inputs, n.n_outputs = 2, 1
        n.inputs[0], n.inputs[1] = self._ref(L["x"]).ptr, self._ref(L["w"]).ptr
        n.outputs[0] = self._ref(L["y"]).ptr
        emit(n, "qnn.conv2d_transpose", [] if L["y"] != op.name else [op.name])
        if L["y"] != op.name:
            transpose_node(L["y"], op.name, self._TO_NHWC, [op.name])

    def _view_ref(self, name: str, shape) -> _lib.TensorRef:
        r = _lib.TensorRef.from_torch(self.buffers[name].view(*shape))
        self._keep.append(r)
        return r

    def _dense_as_conv(self, n, g: ExecGroup, head: PlanOp, ins, outs, emit, stream) -> bool:
        """A dense block [M, K] x [U, K]^T runs as a 1x1 conv block over [M, K, 1, 1]: the NCHW
        output [M, U, 1, 1] is the dense output's memory, requantize/bias stay on axis 1, and
        the conv path's weight packing happens once here instead of padding both operands on
        every run (the dense path's per-call pad_rows kernels).  Records are unchanged (same
        buffers).  Returns False (plain dense block) when the conv would not take MFMA."""
        m, k = head.out.shape[0], self.plan.tensor(head.inputs[0]).shape[1]
        u = head.out.shape[1]
        x4 = self._view_ref(head.inputs[0], (m, k, 1, 1))
        w4 = self._view_ref(head.inputs[1], (u, k, 1, 1))
        ca = n.attrs.block.conv
        ca.strides[:] = [1, 1]
        ca.padding[:] = [0, 0, 0, 0]
        ca.dilation[:] = [1, 1]
        ca.groups = 1
        ca.input_zero_point = head.attrs["input_zero_point"]
        ca.kernel_zero_point = head.attrs["kernel_zero_point"]
        if "kernel_zero_points" in head.consts:
            ca.kernel_zero_points = self._dev_i32(head.consts["kernel_zero_points"]).data_ptr()
        if self.lib.tk_qnn_conv2d_workspace_bytes(x4.ptr, w4.ptr, ctypes.byref(ca)) <= 0:
            n.attrs.block.conv = _lib.tk_conv2d_attrs()
            return False
        # shadow of the input (its producer is a flatten/copy node, which writes none)
        shadow = self._scratch(self.lib.tk_conv2d_shadow_bytes(x4.ptr), zero=True)
        sn = _lib.tk_node()
        sn.kind = _lib.NODE_KINDS["shadow"]
        sn.n_inputs = 1
        sn.inputs[0] = x4.ptr
        sn.n_outputs = 0
        sn.ext[0] = shadow.data_ptr()
        emit(sn, "shadow", [])
        packed = self._scratch(self.lib.tk_conv2d_packed_weight_bytes(w4.ptr, 1))
        sums = self._scratch(((u + 127) // 128 * 128) * 4)
        self._pack(head.inputs[1], head.name, w4, packed, sums, stream)
        n.kind = _lib.NODE_KINDS["conv_block"]
        n.ext[0], n.ext[1], n.ext[2] = shadow.data_ptr(), packed.data_ptr(), sums.data_ptr()
        nbytes = self.lib.tk_conv2d_scratch_bytes(x4.ptr, w4.ptr, ctypes.byref(ca), 1)
        if nbytes < 0:
            _lib.check(-3, f"{head.name} conv scratch")
        if nbytes > 0:
            n.ext[3] = self._scratch(nbytes).data_ptr()
        ins[0], ins[1] = x4, w4
        for i, o in enumerate(g.ops):
            outs[i] = self._view_ref(o.name, tuple(o.out.shape) + (1, 1))
        return True

    def _emit_composite(self, op: PlanOp, mfma, shadow_bufs, ensure_shadow, stream, emit):
        """A tachikoma BYOC composite (relay/contrib/tachikoma.py) = two nodes: the contraction
        with zero zero points into an untraced int32 buffer, then tk_tachikoma_postops writing
        the composite's output (its one trace record, as the reference's composite function is
        one graph node)."""
        torch = _torch()
        acc = torch.empty(op.out.shape, dtype=torch.int32, device=self.device)
        self._keep.append(acc)
        acc_ref = _lib.TensorRef.from_torch(acc)
        self._keep.append(acc_ref)
        ins = [self._ref(op.inputs[0]), self._ref(op.inputs[1])]
        c = _lib.tk_node()
        if op.op == "tachikoma.qnn.conv2d":
            c.kind = _lib.NODE_KINDS["qnn.conv2d"]
            self._conv_attrs(c.attrs.conv2d, op)
            self._prep_conv(c, op, ins, mfma[op.name], shadow_bufs, ensure_shadow, stream)
        else:
            c.kind = _lib.NODE_KINDS["qnn.dense"]
            self._dense_attrs(c.attrs.dense, op)
            c.ext[0] = self._scratch(self.lib.tk_qnn_dense_workspace_bytes(ins[0].ptr, ins[1].ptr)).data_ptr()
        c.n_inputs = 2
        c.inputs[0], c.inputs[1] = ins[0].ptr, ins[1].ptr
        c.n_outputs = 1
        c.outputs[0] = acc_ref.ptr
        emit(c, op.op + ":contraction", [])  # not a record
        p = _lib.tk_node()
        p.kind = _lib.NODE_KINDS["postops"]
        pa = p.attrs.postops
        a = op.attrs
        pa.axis = 1
        pa.clip_lo, pa.clip_hi = a["clip_lo"], a["clip_hi"]
        pa.act_scl, pa.sum_scl, pa.dst_zp = a["act_scl"], a["sum_scl"], a["dst_zp"]
        bias = torch.from_numpy(op.consts["postops_bias"]).to(self.device)
        o_scl = torch.from_numpy(op.consts["postops_o_scl"]).to(self.device)
        self._keep += [bias, o_scl]
        pa.bias, pa.o_scl = bias.data_ptr(), o_scl.data_ptr()
        pa.n_scales = int(o_scl.numel())
        p.n_inputs = 1 + a["has_sum"]
        p.inputs[0] = acc_ref.ptr
        if a["has_sum"]:
            p.inputs[1] = self._ref(op.inputs[2]).ptr
        p.n_outputs = 1
        p.outputs[0] = self._ref(op.name).ptr
        emit(p, op.op, [op.name])

    def _pack(self, param: str, what: str, weight: _lib.TensorRef, packed, sums, stream) -> None:
        """Pack an MFMA conv weight (and its per-channel sums) now, and register the packing
        so that rewriting ``param`` (set_input / load_params) re-derives both."""
        def pack(s: int) -> None:
            _lib.check(self.lib.tk_conv2d_pack_weight(weight.ptr, 1, ctypes.c_void_p(packed.data_ptr()),
                                                      ctypes.c_void_p(sums.data_ptr()), ctypes.c_void_p(s)),
                       f"{what} pack weight")
        pack(stream)
        self._derived.setdefault(param, []).append(pack)

    def _prep_conv(self, n, op: PlanOp, ins, is_mfma: bool, shadow_bufs, ensure_shadow, stream):
        """MFMA path: shadow of the input + packed weight + weight sums (+ scratch: patch sums,
        split-K partial tiles)."""
        if not is_mfma:
            return
        xname = self._conv_io(op)[0]
        ensure_shadow(xname)
        packed = self._scratch(self.lib.tk_conv2d_packed_weight_bytes(ins[1].ptr, 1))
        o = ins[1].shape[0]
        sums = self._scratch(((o + 127) // 128 * 128) * 4)
        self._pack(op.inputs[1], op.name, ins[1], packed, sums, stream)
        n.ext[0] = shadow_bufs[xname].data_ptr()
        n.ext[1] = packed.data_ptr()
        n.ext[2] = sums.data_ptr()
        block = n.kind == _lib.NODE_KINDS["conv_block"]
        ca = n.attrs.block.conv if block else n.attrs.conv2d
        nbytes = self.lib.tk_conv2d_scratch_bytes(ins[0].ptr, ins[1].ptr, ctypes.byref(ca), int(block))
        if nbytes < 0:
            _lib.check(-3, f"{op.name} conv scratch")
        if nbytes > 0:
            n.ext[3] = self._scratch(nbytes).data_ptr()

    @property
    def closed(self) -> bool:
        h = getattr(self, "handle", None)
        return h is None or not h.value

    def close(self) -> None:
        """Release the native module (tk_module_destroy: its HIP graphs, events, streams and packed
        capture mirrors) after the device has finished every stream that may still use them, and
        drop the HBM buffers.  Idempotent.  Runs while the HIP runtime is alive: explicitly, from
        the atexit hook below (before interpreter finalisation and before any library's static
        destructors), or from ``__del__`` outside finalisation -- never from a finaliser at process
        teardown, where the runtime (or a profiler's interception tables) may already be gone."""
        h = getattr(self, "handle", None)
        if h is None or not h.value:
            return
        torch = _torch()
        try:
            torch.cuda.synchronize(self.device)
        finally:
            self.handle = None
            _LIVE.discard(self)
            _lib.check(self.lib.tk_module_destroy(h), "tk_module_destroy")
            self.buffers = {}
            self._keep = []

    def __del__(self):
        if sys.is_finalizing():
            return  # leaked on purpose: the process is ending, no HIP calls from finalisers
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ execution
    def _check_value(self, name: str, value):
        """(host array or device tensor) of ``value`` for buffer ``name``; raises on a shape
        mismatch before anything is written."""
        torch = _torch()
        if name not in self.buffers:
            raise KeyError(f"set_input: {name} is not an input or param of the graph")
        buf = self.buffers[name]
        if isinstance(value, torch.Tensor):
            # held to the exact shape, like host arrays (a transposed or NHWC tensor of the same
            # element count must not be reinterpreted silently)
            if tuple(value.shape) != tuple(buf.shape):
                raise ValueError(f"set_input {name}: shape {tuple(value.shape)} vs {tuple(buf.shape)}")
            return value
        v = np.asarray(value.numpy() if hasattr(value, "numpy") else value)
        if tuple(v.shape) != tuple(buf.shape):
            raise ValueError(f"set_input {name}: shape {v.shape} vs {tuple(buf.shape)}")
        return v

    def set_input(self, name: str, value) -> None:
        """GraphExecutor::SetInput (graph_executor.cc:158-166): copy into the module's buffer on
        the current stream, after the last traced run's copies have read it; a param feeding a
        packed MFMA weight is re-packed."""
        self._write(name, self._check_value(name, value))
        self._rederive([name])

    def set_inputs(self, values: Dict[str, object]) -> None:
        """Several buffers at once, every shape checked before the first write."""
        checked = {k: self._check_value(k, v) for k, v in values.items()}
        for k, v in checked.items():
            self._write(k, v)
        self._rederive(list(checked))

    def _write(self, name: str, v) -> None:
        torch = _torch()
        buf = self.buffers[name]
        s = torch.cuda.current_stream(self.device)
        self.wait_capture(s)
        if isinstance(v, torch.Tensor):
            buf.copy_(v.to(buf.dtype).reshape(buf.shape), non_blocking=True)
        else:
            buf.copy_(torch.from_numpy(np.ascontiguousarray(v.astype(np.dtype(str(buf.dtype).replace("torch.", ""))))))

    def _rederive(self, names: List[str]) -> None:
        s = _lib.stream_handle(_torch().cuda.current_stream(self.device))
        for name in names:
            for fn in self._derived.get(name, []):
                fn(s)

    def wait_capture(self, stream=None) -> None:
        """Make ``stream`` wait for the last traced run's D2H copies (tk_module_wait_capture)."""
        _lib.check(self.lib.tk_module_wait_capture(self.handle, ctypes.c_void_p(_lib.stream_handle(stream))),
                   "tk_module_wait_capture")

    def host_dst_array(self, record_ptrs: Dict[str, int]):
        """Per node × output slot host pointers for tk_module_run (NULL = not captured)."""
        slots = self.n_nodes * _lib.MAX_NODE_OUTPUTS
        arr = (ctypes.c_void_p * slots)()
        for i, recs in enumerate(self.node_records):
            for k, name in enumerate(recs):
                if name in record_ptrs:
                    arr[i * _lib.MAX_NODE_OUTPUTS + k] = record_ptrs[name]
        return arr

    def run(self, stream=None, capture_stream=None, host_dst=None) -> None:
        """One run of every node on ``stream`` (+ the record copies on ``capture_stream`` into
        ``host_dst``).  With ``use_graph`` the run is one replayed HIP graph
        (tk_module_run_graph): the copies then execute inside the launch on ``stream``."""
        s = _lib.stream_handle(stream)
        fn = self.lib.tk_module_run_graph if self.use_graph else self.lib.tk_module_run
        what = "tk_module_run_graph" if self.use_graph else "tk_module_run"
        if host_dst is not None:
            _lib.check(fn(self.handle, ctypes.c_void_p(s), ctypes.c_void_p(_lib.stream_handle(capture_stream)),
                          host_dst), what)
        else:
            _lib.check(fn(self.handle, ctypes.c_void_p(s), None, None), what)

    def run_range(self, begin: int, end: int, stream=None) -> None:
        """Nodes [begin, end) only, on ``stream`` (tk_module_run_range; no capture)."""
        _lib.check(self.lib.tk_module_run_range(self.handle, int(begin), int(end),
                                                ctypes.c_void_p(_lib.stream_handle(stream))), "tk_module_run_range")

    def run_profiled(self, stream=None) -> Dict[str, float]:
        ms = (ctypes.c_float * self.n_nodes)()
        _lib.check(self.lib.tk_module_run_profiled(self.handle, ctypes.c_void_p(_lib.stream_handle(stream)), ms),
                   "tk_module_run_profiled")
        out = {}
        for i, recs in enumerate(self.node_records):
            key = "+".join(recs) if recs else f"<shadow:{i}>"
            out[key] = float(ms[i])
        return out

    def tune(self, max_candidates: int = 16, reps: int = 5, stream=None) -> List[dict]:
        """Find step (tk_module_tune): every MFMA conv-block node keeps the fastest of its first
        ``max_candidates`` kernels, timed on this GPU.  All kernels give bit-identical records.
        Returns (and keeps in ``self.tuning``) per tuned node: records, chosen algo, its time and
        every candidate's."""
        w = max_candidates + 1
        algos = (ctypes.c_int32 * (self.n_nodes * w))()
        us = (ctypes.c_float * (self.n_nodes * w))()
        _lib.check(self.lib.tk_module_tune(self.handle, ctypes.c_void_p(_lib.stream_handle(stream)), max_candidates, reps,
                                           algos, us), "tk_module_tune")
        out = []
        for i in range(self.n_nodes):
            if algos[i * w] < 0:
                continue
            cands = [(int(algos[i * w + 1 + c]), round(float(us[i * w + 1 + c]), 2)) for c in range(max_candidates)
                     if algos[i * w + 1 + c] >= 0]
            out.append({"node": i, "records": list(self.node_records[i]), "algo": int(algos[i * w]),
                        "us": round(float(us[i * w]), 2), "kernel": self.algo_info(i, int(algos[i * w])),
                        "candidates": cands})
        self.tuning = out
        self.tune_table_digest = tune_table_digest(out)
        return out

    def tuning_table(self) -> dict:
        """The find step's choice per conv-block node, keyed by the node's records (stable across
        processes for one plan), with the library it was measured with."""
        return {"format": "tachikoma-tune-table", "version": 2, "library": _lib.build_info(),
                "entries": [{"records": t["records"], "algo": t["algo"], "us": t["us"],
                             "kernel": t.get("kernel") or self.algo_info(t["node"], t["algo"])} for t in self.tuning]}

    def apply_tuning(self, table) -> List[dict]:
        """Replays a tune table (``tuning_table()``, or a JSON file of one) with tk_module_set_node_algo;
        every conv-block node must be listed.  Returns (and keeps in ``self.tuning``) the applied
        entries; the table's digest is ``self.tune_table_digest``."""
        import json
        if isinstance(table, str):
            with open(table) as f:
                table = json.load(f)
        if table.get("format") != "tachikoma-tune-table":
            raise _lib.TachikomaError("not a tachikoma tune table")
        by_records = {tuple(e["records"]): e for e in table["entries"]}
        same_lib = table.get("library") == _lib.build_info()
        applied = []
        for i, (kind, recs) in enumerate(zip(self.node_kinds, self.node_records)):
            if self._node_kind(i) != _lib.NODE_KINDS["conv_block"]:  # dense blocks run as 1x1 conv blocks
                continue
            e = by_records.get(tuple(recs))
            if e is None:
                raise _lib.TachikomaError(f"tune table has no entry for the conv block writing {recs}")
            # algo numbers are plan indices that move when the planner changes: a table from another
            # library is replayed by kernel description (version 2 tables), never by number
            algo = int(e["algo"])
            if algo == 0:
                pass  # the library's own choice (blocks with no kernel list, e.g. depthwise): no description to match
            elif e.get("kernel"):
                if not (same_lib and self.algo_info(i, algo) == e["kernel"]):
                    match = [a for a in self.node_algos(i) if self.algo_info(i, a) == e["kernel"]]
                    if not match:
                        raise _lib.TachikomaError(f"tune table: no kernel '{e['kernel']}' for the conv block "
                                                  f"writing {recs} in this library")
                    algo = match[0]
            elif not same_lib:
                raise _lib.TachikomaError(f"tune table from library {table.get('library')} (this is "
                                          f"{_lib.build_info()}) has no kernel descriptions: algo numbers would "
                                          f"select other kernels")
            _lib.check(self.lib.tk_module_set_node_algo(self.handle, i, algo), "tk_module_set_node_algo")
            applied.append({"node": i, "records": list(recs), "algo": algo, "us": e.get("us"),
                            "kernel": self.algo_info(i, algo), "candidates": []})
        self.tuning = applied
        self.tune_table_digest = tune_table_digest(applied)
        return applied

    def node_algos(self, node: int) -> List[int]:
        """tk_conv2d_block_algos: every kernel (algo) conv-block node `node` can run on."""
        n = self._nodes[node]
        buf = (ctypes.c_int32 * 512)()
        cnt = self.lib.tk_conv2d_block_algos(n.inputs[0], n.inputs[1], ctypes.byref(n.attrs.block), buf, 512)
        _lib.check(min(cnt, 0), "tk_conv2d_block_algos")
        return list(buf[:min(cnt, 512)])

    def algo_info(self, node: int, algo: int) -> str:
        """tk_conv2d_block_algo_info: what kernel `algo` is on conv-block node `node`."""
        n = self._nodes[node]
        buf = ctypes.create_string_buffer(256)
        rc = self.lib.tk_conv2d_block_algo_info(n.inputs[0], n.inputs[1], ctypes.byref(n.attrs.block), int(algo), buf,
                                               len(buf))
        return buf.value.decode() if rc == 0 else f"algo {algo} (not listed)"

    def _node_kind(self, i: int) -> int:
        return self._node_kind_codes[i]

    def set_copy_trace(self, enable: bool) -> None:
        """Per-chunk copy timing of packed traced runs (tk_module_set_copy_trace)."""
        _lib.check(self.lib.tk_module_set_copy_trace(self.handle, int(enable)), "tk_module_set_copy_trace")

    def copy_trace(self) -> List[dict]:
        """The last packed traced run's chunk copies: bytes, start / end ms after the run's first
        launch (tk_module_copy_trace; waits for those copies)."""
        n = self.lib.tk_module_copy_trace(self.handle, None, 0)
        _lib.check(min(n, 0), "tk_module_copy_trace")
        buf = (ctypes.c_double * max(1, 3 * n))()
        _lib.check(min(self.lib.tk_module_copy_trace(self.handle, buf, n), 0), "tk_module_copy_trace")
        return [{"bytes": int(buf[3 * c]), "start_ms": buf[3 * c + 1], "end_ms": buf[3 * c + 2]} for c in range(n)]

    def set_profiling(self, enable: bool) -> None:
        _lib.check(self.lib.tk_module_set_profiling(self.handle, int(enable)), "tk_module_set_profiling")

    def node_times(self) -> List[float]:
        ms = (ctypes.c_float * self.n_nodes)()
        _lib.check(self.lib.tk_module_node_times(self.handle, ms), "tk_module_node_times")
        return [float(v) for v in ms]

    def records_digest(self, stream=None):
        """Device digest of every trace record (trace_format.records_digest twin), enqueued on
        ``stream``; returns a 1-element int64 device tensor (the u64 digest's bit pattern)."""
        torch = _torch()
        recs = self.plan.records
        if getattr(self, "_digest_slots", None) is None:
            self._digest_slots = torch.zeros(max(1, len(recs)), dtype=torch.int64, device=self.device)
            self._digest_out = torch.zeros(1, dtype=torch.int64, device=self.device)
        s = ctypes.c_void_p(_lib.stream_handle(stream))
        base = self._digest_slots.data_ptr()
        for i, t in enumerate(recs):
            buf = self.buffers[t.name]
            _lib.check(self.lib.tk_digest_bytes(ctypes.c_void_p(buf.data_ptr()), buf.numel() * buf.element_size(),
                                                ctypes.c_void_p(base + 8 * i), s), f"digest {t.name}")
        _lib.check(self.lib.tk_digest_bytes(ctypes.c_void_p(base), 8 * len(recs),
                                            ctypes.c_void_p(self._digest_out.data_ptr()), s), "digest")
        return self._digest_out

    def output(self, name: str):
        return self.buffers[name]


def _fill_qnn_add(qa, a) -> None:
    """tk_qnn_add_attrs from a lowered qnn.add (per-tensor RequantizeOrUpcast per side)."""
    for side in ("lhs", "rhs"):
        r = getattr(qa, side)
        r.mode = a[f"{side}_mode"]
        r.axis = -1
        r.multiplier = a[f"{side}_multiplier"]
        r.shift = a[f"{side}_shift"]
        r.input_zero_point = a[f"{side}_zero_point"]
        r.output_zero_point = a["output_zero_point"]
    qa.output_zero_point = a["output_zero_point"]
    qa.lhs_upcast = a["lhs_upcast"]
    qa.rhs_upcast = a["rhs_upcast"]


def _as_torch_device(dev):
    torch = _torch()
    if isinstance(dev, torch.device):
        return dev
    if isinstance(dev, int):
        return torch.device("cuda", dev)
    if hasattr(dev, "device_id"):
        return torch.device("cuda", int(dev.device_id))
    return torch.device(dev)

"""Relay text format for the QNN subset: ``parse`` (tvm.parser.parse, src/parser/parser.cc)
and ``astext`` (IRModule.astext, src/printer/relay_text_printer.cc).

Accepted text is what ``mod.astext()`` prints for integer QNN graphs::

    #[version = "0.0.5"]
    def @main(%data: Tensor[(1, 3, 224, 224), int8], %w: Tensor[(64, 3, 7, 7), int8]) {
      %0 = qnn.conv2d(%data, %w, 0, 0, 0.0235f, meta[relay.Constant][0], padding=[3, 3, 3, 3],
                      channels=64, kernel_size=[7, 7], out_dtype="int32") /* ty=Tensor[...] */;
      ...
    }
    #[metadata]
    {"root": 1, "nodes": [...], "b64ndarrays": [...], "attrs": {"tvm_version": "0.11.dev0"}}

* literals: ``3`` (int32), ``3i64`` / ``3i8`` / ``3u8``, ``0.5f`` / ``1f32`` / ``2f64``, strings,
  ``[..]`` / ``(..)`` sequences, ``True``/``False``/``None``;
* ``meta[relay.Constant][i]``: the i-th constant of the metadata section — a JSON node graph
  (src/node/serialization.cc:470-530) whose tensors are base64 ``SaveDLTensor`` blobs
  (include/tvm/runtime/ndarray.h:447-494) — or of ``init_meta_table``;
* ``/* ... */`` (type annotations) and ``// ...`` comments are skipped.

Ops map onto this package's constructors (``relay.qnn.op.*``, ``relay.nn.*``), which take the
reference's attribute names; anything else raises ``ParseError``.  Float models as the reference's
own tests write them (``nn.batch_norm`` with its ``%k.0`` field projection, ``nn.pad`` with the
pad value as an argument, ``reshape`` with 0 / -1) parse too: tests/golden/menangerie_*.relay.
"""
from __future__ import annotations

import base64
import json
import re
import struct
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import op as _op
from .expr import Call, Constant, Expr, Function, IRModule, Tuple, Var, const, post_order
from .qnn import op as _qnn

__all__ = ["ParseError", "parse", "fromtext", "astext", "load_meta_json", "dump_meta_json"]


class ParseError(ValueError):
    pass


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<lcomment>//[^\n]*)
  | (?P<bcomment>/\*.*?\*/)
  | (?P<attr>\#\[[^\]]*\])
  | (?P<string>"(?:[^"\\]|\\.)*")
  | (?P<number>-?(?:\d+\.\d*(?:[eE][-+]?\d+)?|\d*\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?)(?:f(?:16|32|64)?|i(?:8|16|32|64)|u(?:8|16|32|64))?)
  | (?P<local>%[A-Za-z0-9_.]+)
  | (?P<global>@[A-Za-z0-9_.]+)
  | (?P<arrow>->)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_.]*)
  | (?P<punct>[()\[\]{},=:;])
""", re.VERBOSE | re.DOTALL)


def _tokenize(src: str) -> List[Tuple[str, str]]:
    toks, pos = [], 0
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise ParseError(f"unexpected character {src[pos]!r} at offset {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "lcomment", "bcomment", "attr"):
            continue
        toks.append((kind, m.group()))
    toks.append(("eof", ""))
    return toks


_NUM_SUFFIX = re.compile(r"^(?P<v>-?[0-9.eE+-]+?)(?P<s>f(?:16|32|64)?|i(?:8|16|32|64)|u(?:8|16|32|64))?$")


def _number(text: str):
    m = _NUM_SUFFIX.match(text)
    v, s = m.group("v"), m.group("s")
    if s is None:
        if any(c in v for c in ".eE"):
            return np.float32(float(v))
        return np.int32(int(v))
    if s[0] == "f":
        return np.dtype("float" + (s[1:] or "32")).type(float(v))
    kind = "int" if s[0] == "i" else "uint"
    return np.dtype(kind + s[1:]).type(int(float(v)))


# ---------------------------------------------------------------- metadata section

def _load_dltensor(blob: bytes) -> np.ndarray:
    """One ``SaveDLTensor`` record (ndarray.h:447-494)."""
    magic, _reserved = struct.unpack_from("<QQ", blob, 0)
    if magic != 0xDD5E40F096B4A13F:
        raise ParseError("metadata tensor: bad NDArray magic")
    _dev_type, _dev_id, ndim = struct.unpack_from("<iii", blob, 16)
    code, bits, lanes = struct.unpack_from("<BBH", blob, 28)
    shape = struct.unpack_from(f"<{ndim}q", blob, 32) if ndim else ()
    off = 32 + 8 * ndim
    (nbytes,) = struct.unpack_from("<q", blob, off)
    kind = {0: "i", 1: "u", 2: "f"}.get(code)
    if kind is None or lanes != 1:
        raise ParseError(f"metadata tensor: unsupported dtype code {code} lanes {lanes}")
    dt = np.dtype(f"<{kind}{bits // 8}")
    return np.frombuffer(blob, dtype=dt, count=nbytes // dt.itemsize, offset=off + 8).reshape(shape).copy()


def load_meta_json(text: str) -> Dict[str, List[Any]]:
    """The metadata map {"relay.Constant": [np.ndarray, ...]} of a ``#[metadata]`` section."""
    g = json.loads(text)
    nodes, arrays = g["nodes"], [base64.b64decode(b) for b in g.get("b64ndarrays", [])]

    def value(idx: int):
        node = nodes[idx]
        key = node.get("type_key", "")
        if key == "relay.Constant":
            return _load_dltensor(arrays[int(node["attrs"]["data"])])
        if key == "Array":
            return [value(i) for i in node.get("data", [])]
        if key == "Map":
            if node.get("keys"):
                return {k: value(i) for k, i in zip(node["keys"], node["data"])}
            d = node.get("data", [])
            return {value(d[i]): value(d[i + 1]) for i in range(0, len(d), 2)}
        if key in ("runtime.String", "String"):
            return node.get("repr_str", node.get("attrs", {}).get("data", ""))
        return None

    root = value(int(g["root"]))
    if not isinstance(root, dict):
        raise ParseError("metadata root must be a map")
    return root


def dump_meta_json(constants: List[np.ndarray]) -> str:
    """Metadata section holding ``constants`` as meta[relay.Constant][i] (serialization.cc layout)."""
    nodes: List[dict] = [{"type_key": ""}, {"type_key": "Map", "keys": ["relay.Constant"], "data": [2]},
                         {"type_key": "Array", "data": [3 + i for i in range(len(constants))]}]
    b64 = []
    for i, c in enumerate(constants):
        c = np.ascontiguousarray(c)
        code = {"i": 0, "u": 1, "f": 2}[c.dtype.kind]
        head = struct.pack("<QQiii", 0xDD5E40F096B4A13F, 0, 1, 0, c.ndim) + struct.pack("<BBH", code,
                                                                                         c.dtype.itemsize * 8, 1)
        head += struct.pack(f"<{c.ndim}q", *c.shape) + struct.pack("<q", c.nbytes)
        b64.append(base64.b64encode(head + c.tobytes()).decode())
        nodes.append({"type_key": "relay.Constant", "attrs": {"data": str(i), "span": "0",
                                                              "virtual_device_": "0", "_checked_type_": "0"}})
    return json.dumps({"root": 1, "nodes": nodes, "b64ndarrays": b64, "attrs": {"tvm_version": "0.11.dev0"}})


# ---------------------------------------------------------------- parser

def _call(op: str, args: List[Expr], attrs: Dict[str, Any]) -> Expr:
    def seq(v):
        return tuple(v) if isinstance(v, (list, tuple)) else v
    a = {k: seq(v) for k, v in attrs.items()}
    try:
        if op == "qnn.conv2d":
            return _qnn.conv2d(*args, **a)
        if op == "qnn.dense":
            return _qnn.dense(*args, **a)
        if op == "qnn.requantize":
            return _qnn.requantize(*args, **a)
        if op in ("qnn.add", "qnn.subtract", "qnn.mul", "qnn.concatenate", "qnn.quantize", "qnn.dequantize",
                  "qnn.leaky_relu", "qnn.batch_matmul", "qnn.conv2d_transpose") or op in _qnn.UNARY_OPS:
            if op == "qnn.batch_matmul":
                a.pop("transpose_a", None)
                a.pop("transpose_b", None)
            if op == "qnn.leaky_relu":  # alpha is an attribute, the constructor's second argument
                return _qnn.leaky_relu(args[0], a.pop("alpha"), *args[1:], **a)
            return getattr(_qnn, op.split(".")[1])(*args, **a)
        if op in ("qnn.simulated_quantize", "qnn.simulated_dequantize"):
            return _qnn.simulated_call(op, *args, **a)
        if op == "transpose":
            return _op.transpose(*args, **a)
        if op == "nn.bias_add":
            return _op.bias_add(*args, **a)
        if op == "clip":
            return _op.clip(*args, **a)
        if op == "nn.relu":
            return _op.relu(*args)
        if op == "cast":
            return _op.cast(*args, **a)
        if op == "nn.max_pool2d":
            return _op.max_pool2d(*args, **a)
        if op == "nn.avg_pool2d":
            return _op.avg_pool2d(*args, **a)
        if op == "nn.global_avg_pool2d":
            return _op.global_avg_pool2d(*args, **a)
        if op == "nn.batch_flatten":
            return _op.batch_flatten(*args)
        if op == "reshape":
            return _op.reshape(*args, **a)
        # float models as the reference's own tests write them (tests/python/relay/collage/
        # menangerie.py): batch norm layers and explicit padding
        if op == "nn.batch_norm":
            return _op.batch_norm(*args, **a)
        if op == "nn.pad":
            return _op.pad(args[0], a.pop("pad_width"), *args[1:], **a)
        # float32 graphs and relay.quantize-realized graphs
        if op == "nn.conv2d":
            return _op.conv2d(*args, **a)
        if op == "nn.dense":
            return _op.dense(*args, **a)
        if op in ("add", "multiply", "right_shift", "left_shift"):
            return getattr(_op, op)(*args)
        if op == "round":
            return _op.round(*args)
        if op == "fixed_point_multiply":
            return _op.fixed_point_multiply(*args, **a)
        if op == "annotation.stop_fusion":
            return _op.stop_fusion(*args)
        if op == "annotation.cast_hint":
            return _op.cast_hint(*args, **a)
        if op == "relay.op.annotation.simulated_quantize":
            from .quantize.passes import simulated_quantize
            return simulated_quantize(*args, **a)
    except TypeError as e:
        raise ParseError(f"{op}: {e}") from e
    raise ParseError(f"operator {op} is not in the supported subset (QNN, float32 CNN, realized quantized graphs)")


class _Parser:
    def __init__(self, src: str, meta: Optional[Dict[str, List[Any]]]):
        # split off the metadata section first (its JSON is not Relay tokens)
        body, _, meta_text = src.partition("#[metadata]")
        self.meta = dict(meta or {})
        if meta_text.strip():
            self.meta.update(load_meta_json(meta_text.strip()))
        self.toks = _tokenize(body)
        self.i = 0
        self.scope: Dict[str, Expr] = {}

    def peek(self, k=0):
        return self.toks[self.i + k]

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def expect(self, text):
        t = self.next()
        if t[1] != text:
            raise ParseError(f"expected {text!r}, got {t[1]!r}")
        return t

    def parse_module(self) -> IRModule:
        main = None
        while self.peek()[0] != "eof":
            t = self.next()
            if t != ("ident", "def"):
                raise ParseError(f"expected 'def', got {t[1]!r}")
            name = self.next()
            fn = self.parse_function()
            if name[1] == "@main":
                main = fn
        if main is None:
            raise ParseError("no @main function")
        return IRModule(main)

    def parse_type(self):
        t = self.next()
        if t == ("ident", "Tensor"):
            self.expect("[")
            self.expect("(")
            dims = []
            while self.peek()[1] != ")":
                dims.append(int(self.next()[1]))
                if self.peek()[1] == ",":
                    self.next()
            self.expect(")")
            self.expect(",")
            dtype = self.next()[1]
            self.expect("]")
            return tuple(dims), dtype
        if t[0] == "ident":
            return (), t[1]
        raise ParseError(f"bad type {t[1]!r}")

    def parse_function(self) -> Function:
        self.expect("(")
        params = []
        while self.peek()[1] != ")":
            name = self.next()
            if name[0] != "local":
                raise ParseError(f"expected a parameter, got {name[1]!r}")
            self.expect(":")
            shape, dtype = self.parse_type()
            v = Var(name[1][1:], shape, dtype)
            self.scope[name[1]] = v
            params.append(v)
            if self.peek()[1] == ",":
                self.next()
        self.expect(")")
        if self.peek()[0] == "arrow":
            self.next()
            self.parse_type()
        self.expect("{")
        body = None
        while self.peek()[1] != "}":
            if self.peek()[0] == "local" and self.peek(1)[1] == "=":
                name = self.next()[1]
                self.next()
                self.scope[name] = self.parse_expr()
                self.expect(";")
            else:
                body = self.parse_expr()
                if self.peek()[1] == ";":
                    self.next()
        self.expect("}")
        if body is None:
            raise ParseError("function has no result expression")
        return Function(params, body)

    def parse_value(self):
        """Attribute / literal value (python object)."""
        t = self.peek()
        if t[1] in ("[", "("):
            close = "]" if t[1] == "[" else ")"
            self.next()
            out = []
            while self.peek()[1] != close:
                out.append(self.parse_value())
                if self.peek()[1] == ",":
                    self.next()
            self.next()
            return out
        self.next()
        if t[0] == "string":
            return json.loads(t[1])
        if t[0] == "number":
            m = _NUM_SUFFIX.match(t[1])
            if m.group("s") is None and any(c in m.group("v") for c in ".eE"):
                return float(m.group("v"))  # a double attribute (e.g. qnn.leaky_relu's alpha), not float32
            v = _number(t[1])
            return v.item()
        if t[1] in ("True", "False"):
            return t[1] == "True"
        if t[1] == "None":
            return None
        return t[1]

    def parse_expr(self) -> Expr:
        t = self.peek()
        if t[0] == "local":
            self.next()
            name = t[1]
            if name not in self.scope:
                # a tuple field (TupleGetItem, ``%0.0``)
                base, dot, idx = name.rpartition(".")
                if dot and idx.isdigit() and base in self.scope:
                    tup = self.scope[base]
                    if isinstance(tup, Tuple):
                        if int(idx) >= len(tup):
                            raise ParseError(f"{name}: {base} has {len(tup)} fields")
                        return tup[int(idx)]
                    if not isinstance(tup, _op.BatchNormOutputs):
                        raise ParseError(f"{name}: {base} is not a tuple")
                    try:
                        return tup[int(idx)]
                    except NotImplementedError as e:
                        raise ParseError(f"{name}: {e}") from e
                raise ParseError(f"unbound variable {name}")
            v = self.scope[name]
            if isinstance(v, _op.BatchNormOutputs):
                raise ParseError(f"{name} is a tuple (nn.batch_norm): use a field, e.g. {name}.0")
            return v
        if t[1] == "(":
            # a tuple literal -- qnn.concatenate's tensors, scales and zero points: `()`, `(a,)` or
            # two or more fields -- or a parenthesised expression `(a)` (grouping, not a 1-tuple)
            self.next()
            fields = []
            comma = False
            while self.peek()[1] != ")":
                fields.append(self.parse_expr())
                if self.peek()[1] == ",":
                    self.next()
                    comma = True
            self.next()
            if len(fields) == 1 and not comma:
                return fields[0]
            return Tuple(fields)
        if t[0] == "number":
            self.next()
            v = _number(t[1])
            return const(v, str(np.asarray(v).dtype))
        if t == ("ident", "meta"):
            self.next()
            self.expect("[")
            kind = self.next()[1]
            self.expect("]")
            self.expect("[")
            idx = int(self.next()[1])
            self.expect("]")
            if kind != "relay.Constant" or kind not in self.meta or idx >= len(self.meta[kind]):
                raise ParseError(f"meta[{kind}][{idx}] is not in the metadata")
            return Constant(np.asarray(self.meta[kind][idx]))
        if t[0] == "ident":
            op = self.next()[1]
            self.expect("(")
            args, attrs = [], {}
            while self.peek()[1] != ")":
                if self.peek()[0] == "ident" and self.peek(1)[1] == "=":
                    key = self.next()[1]
                    self.next()
                    attrs[key] = self.parse_value()
                else:
                    args.append(self.parse_expr())
                if self.peek()[1] == ",":
                    self.next()
            self.expect(")")
            return _call(op, args, attrs)
        raise ParseError(f"unexpected token {t[1]!r}")


def parse(source: str, source_name: str = "from_string", init_module=None,
          init_meta_table: Optional[Dict[str, List[Any]]] = None) -> IRModule:
    """``tvm.parser.parse`` for the integer QNN subset (src/parser/parser.cc)."""
    if init_module is not None:
        raise ParseError("init_module is not supported")
    return _Parser(source, init_meta_table).parse_module()


def fromtext(source: str, source_name: str = "from_string") -> IRModule:
    return parse(source, source_name)


# ---------------------------------------------------------------- printer

def _fmt_value(v) -> str:
    if isinstance(v, bool):
        return "True" if v else "False"
    if v is None:
        return "None"
    if isinstance(v, str):
        return json.dumps(v)
    if isinstance(v, (list, tuple)):
        return "[" + ", ".join(_fmt_value(x) for x in v) + "]"
    if isinstance(v, float):
        return repr(v)
    return str(v)


def _fmt_const(c: Constant, metas: List[np.ndarray]) -> str:
    d = c.data
    if d.ndim == 0:
        if d.dtype == np.float32:
            return f"{float(d)!r}f"
        if d.dtype == np.int32:
            return str(int(d))
        suffix = {"f": "f", "i": "i", "u": "u"}[d.dtype.kind] + str(d.dtype.itemsize * 8)
        return f"{d.item()!r}{suffix}"
    metas.append(d)
    return f"meta[relay.Constant][{len(metas) - 1}]"


_DEFAULT_ATTRS = {"cfg_rounding", "cfg_compute_dtype"}


def astext(mod: IRModule, show_meta_data: bool = True) -> str:
    """``IRModule.astext``: calls numbered %0, %1, ... in post-order (the MRT names)."""
    fn = mod["main"]
    names: Dict[int, str] = {}
    metas: List[np.ndarray] = []
    lines = []
    counter = 0

    def ref(e: Expr) -> str:
        if isinstance(e, Var):
            return "%" + e.name_hint
        if isinstance(e, Constant):
            return _fmt_const(e, metas)
        if isinstance(e, Tuple):  # printed inline: it takes no %N (no record, no MRT symbol)
            return "(" + ", ".join(ref(f) for f in e.fields) + ("," if len(e.fields) == 1 else "") + ")"
        return names[id(e)]

    for node in post_order(fn.body):
        if not isinstance(node, Call):
            continue
        args = [ref(a) for a in node.args]
        attrs = [f"{k}={_fmt_value(v)}" for k, v in node.attrs.items()
                 if k not in _DEFAULT_ATTRS and not (k in ("rounding", "compute_dtype") and v == "None")]
        ty = f"Tensor[({', '.join(map(str, node.shape))}{',' if len(node.shape) == 1 else ''}), {node.dtype}]"
        names[id(node)] = f"%{counter}"
        lines.append(f"  %{counter} = {node.op}({', '.join(args + attrs)}) /* ty={ty} */;")
        counter += 1
        if node.op == "nn.batch_norm":  # a tuple: consumers read its field 0 (a TupleGetItem line)
            lines.append(f"  %{counter} = %{counter - 1}.0 /* ty={ty} */;")
            names[id(node)] = f"%{counter}"
            counter += 1
    params = ", ".join(f"%{p.name_hint}: Tensor[({', '.join(map(str, p.shape))}{',' if len(p.shape) == 1 else ''}), "
                       f"{p.dtype}]" for p in fn.params)
    body_ref = ref(fn.body)
    if lines and lines[-1].startswith(f"  {body_ref} = "):
        last = lines.pop()
        lines.append("  " + last.split(" = ", 1)[1].rstrip(";"))
    else:
        lines.append(f"  {body_ref}")
    text = '#[version = "0.0.5"]\n' + f"def @main({params}) {{\n" + "\n".join(lines) + "\n}\n"
    if show_meta_data and metas:
        text += "\n#[metadata]\n" + dump_meta_json(metas) + "\n"
    return text

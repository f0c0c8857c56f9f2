"""FuseOps grouping and fused-function naming over a lowered plan.

The reference's graph executor runs *fused* primitive functions, and its debug executor
dumps one tensor per fused node.  This module reproduces how those
nodes come about, on this engine's plan:

* ``fuse_ops`` — the partitioner of src/relay/transforms/fuse_ops.cc: an indexed forward
  graph in post-DFS order (:98-330), its post-dominator tree by least common ancestors
  (:380-510), and the three ``RunFuse`` phases (:705-800) with ``CheckPath`` /
  ``CommitFuse`` / union-find groups (:572-700) and ``relay.FuseOps.max_depth`` (:84-89,
  default 256).  Op patterns are those of the ops the plan's QNN ops canonicalise to:
  contractions and pools are kOutEWiseFusable anchors, requantize / clip / cast are
  elementwise, bias_add and qnn.add broadcast (elementwise on same-shape edges), flatten /
  reshape injective.
* ``function_names`` — te_compiler_cache.cc:222-236 (``"fused"`` + ``_<op name>`` per call in
  post order, truncated at 80 characters with ``_<hex std::hash>_``), prefixed
  ``tvmgen_<mod_name>`` and made unique by name_supply.cc:46-91 (``.`` → ``_``, ``_1``, ``_2``
  suffixes); structurally equal groups share one function, as the TE compiler cache does
  (te_compiler.cc:355-400).
* graph node names — graph_executor_codegen.cc:462-465 (``FreshName(func_name)`` per call).

Granularity note: the reference fuses *after* QNN canonicalisation, so its functions also
hold the int16 casts / zero-point subtractions that precede each conv; here the groups are
formed over the QNN-level ops the trace records, with the same algorithm.
"""
from __future__ import annotations

import hashlib
import json
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

# OpPatternKind (include/tvm/relay/op_attr_types.h)
kElemWise, kBroadcast, kInjective, kCommReduce, kOutEWiseFusable, kTuple, kOpaque = 0, 1, 2, 3, 4, 7, 8
MAX_FUSED_OPS = 256            # kMaxFusedOps, fuse_ops.cc
MAX_FUNC_NAME_LENGTH = 80      # kMaxFuncNameLength, te_compiler_cache.cc:228

_PATTERNS = {
    "qnn.conv2d": kOutEWiseFusable, "qnn.dense": kOutEWiseFusable, "nn.conv2d": kOutEWiseFusable,
    "nn.dense": kOutEWiseFusable, "nn.max_pool2d": kOutEWiseFusable, "nn.avg_pool2d": kOutEWiseFusable,
    "nn.global_avg_pool2d": kOutEWiseFusable,
    "qnn.requantize": kElemWise, "clip": kElemWise, "cast": kElemWise, "nn.relu": kElemWise,
    "round": kElemWise, "fixed_point_multiply": kElemWise,
    "nn.bias_add": kBroadcast, "qnn.add": kBroadcast, "add": kBroadcast, "multiply": kBroadcast,
    "left_shift": kBroadcast, "right_shift": kBroadcast, "subtract": kBroadcast,
    "fixed_point_multiply_per_axis": kBroadcast,  # transform.cc:4421-4432
    "greater_equal": kBroadcast, "where": kBroadcast,  # TONEAREST requantize (FixedPointMultiplyToNearest)
    "nn.batch_flatten": kInjective, "reshape": kInjective, "nn.pad": kInjective,
    # pre-quantized graphs: the pattern of each op's canonical form (divide / round / add / clip /
    # cast; cast / subtract / multiply; requantizes + subtract / multiply; requantizes + concatenate)
    "qnn.quantize": kBroadcast, "qnn.dequantize": kBroadcast, "qnn.subtract": kBroadcast, "qnn.mul": kBroadcast,
    "qnn.concatenate": kInjective, "transpose": kInjective,
    # round 5: leaky_relu canonicalizes to requantize / fixed_point_multiply / add / where (broadcast),
    # the unary ops to take (injective), batch_matmul / conv2d_transpose to their nn ops
    "qnn.leaky_relu": kBroadcast, "qnn.batch_matmul": kOutEWiseFusable, "qnn.conv2d_transpose": kOutEWiseFusable,
    **{f"qnn.{u}": kInjective for u in ("sqrt", "rsqrt", "exp", "erf", "sigmoid", "hardswish", "tanh", "log", "abs")},
    # the simulated ops register OpPattern.ELEMWISE themselves (relay/qnn/op/_qnn.py:39,53)
    "qnn.simulated_quantize": kElemWise, "qnn.simulated_dequantize": kElemWise,
    "annotation.stop_fusion": kOpaque, "annotation.cast_hint": kOpaque,
    "tachikoma.qnn.conv2d": kOpaque, "tachikoma.qnn.dense": kOpaque,  # external (BYOC) functions
}


def relay_op_name(op) -> str:
    """The Relay operator a plan op came from (lowering renames a few: ewise, bias_add)."""
    return op.attrs.get("relay_op", op.op)


def op_pattern(op) -> int:
    return _PATTERNS.get(relay_op_name(op), kOpaque)


# ---------------------------------------------------------------- the partitioner

class _Node:
    __slots__ = ("name", "index", "extern_ref", "pattern", "outputs")

    def __init__(self, name: str):
        self.name = name
        self.index = 0
        self.extern_ref = False
        self.pattern = kOpaque
        self.outputs: List[Tuple["_Node", int]] = []  # (consumer, edge pattern)


class _DomNode:
    __slots__ = ("gnode", "parent", "depth", "pattern")

    def __init__(self, gnode):
        self.gnode = gnode
        self.parent: Optional["_DomNode"] = None
        self.depth = 0
        self.pattern = kOpaque


class _Group:
    __slots__ = ("parent", "pattern", "root", "anchor", "num_nodes")

    def __init__(self, pattern: int, root: str, anchor: Optional[str]):
        self.parent: Optional["_Group"] = None
        self.pattern = pattern
        self.root = root
        self.anchor = anchor
        self.num_nodes = 1

    def find_root(self) -> "_Group":
        root = self
        while root.parent is not None:
            root = root.parent
        p = self
        while p is not root:
            nxt = p.parent
            p.parent = root
            p = nxt
        return root


def _forward_graph(plan) -> List[_Node]:
    """IndexedForwardGraph::Creator over the plan: variables and ops in post-DFS order; the
    function's params and its result are referenced externally (fuse_ops.cc:160-290)."""
    shapes = {t.name: tuple(t.shape) for t in list(plan.inputs) + list(plan.params)}
    for op in plan.ops:
        shapes[op.name] = tuple(op.out.shape)
    nodes: Dict[str, _Node] = {}
    order: List[_Node] = []

    def node(name):
        if name not in nodes:
            nodes[name] = _Node(name)
        return nodes[name]

    op_names = {op.name for op in plan.ops}
    for op in plan.ops:
        for x in op.inputs:
            if x not in op_names and x not in nodes:
                n = node(x)           # a function param: visited where first used
                n.extern_ref = True
                n.index = len(order)
                order.append(n)
        me = node(op.name)
        pat = op_pattern(op)
        me.pattern = pat
        for x in op.inputs:
            edge = pat
            if edge == kBroadcast and shapes.get(x) == tuple(op.out.shape):
                edge = kElemWise
            nodes[x].outputs.insert(0, (me, edge))  # LinkedList::Push prepends
        me.index = len(order)
        order.append(me)
    for o in plan.outputs:
        nodes[o].extern_ref = True
    return order


def _post_dom(order: List[_Node]) -> List[_DomNode]:
    tree: List[Optional[_DomNode]] = [None] * len(order)

    def lca(a, b, pat):
        while a is not b:
            if a is None or b is None:
                return None, pat
            if a.depth < b.depth:
                pat = max(pat, b.pattern)
                b = b.parent
            elif b.depth < a.depth:
                pat = max(pat, a.pattern)
                a = a.parent
            else:
                pat = max(pat, a.pattern, b.pattern)
                a, b = a.parent, b.parent
        return a, pat

    for i in range(len(order) - 1, -1, -1):
        g = order[i]
        t = _DomNode(g)
        if g.extern_ref:
            t.depth, t.parent, t.pattern = 1, None, kOpaque
        else:
            pat = kElemWise
            parent = None
            if g.outputs:
                first, epat = g.outputs[0]
                parent = tree[first.index]
                pat = max(pat, epat)
                for cons, epat in g.outputs[1:]:
                    parent, pat = lca(parent, tree[cons.index], pat)
                    pat = max(pat, epat)
            t.depth = parent.depth + 1 if parent is not None else 1
            t.parent = parent
            t.pattern = pat
        tree[i] = t
    return tree


def _combine(lhs: int, rhs: int) -> int:
    if lhs > kBroadcast and rhs > kBroadcast:
        raise RuntimeError("Cannot merge two complex group together")
    return max(lhs, rhs)


def partition(plan, opt_level: int = 3, max_depth: int = MAX_FUSED_OPS) -> Dict[str, _Group]:
    """GraphPartitioner::Partition: {node name: root group}."""
    order = _forward_graph(plan)
    groups = [_Group(n.pattern, n.name, n.name if n.pattern == kOutEWiseFusable else None) for n in order]
    if opt_level == 0:
        return {n.name: groups[n.index] for n in order}
    tree = _post_dom(order)

    def check_path(src, sink, fcond):
        visited = set()

        def rec(n):
            if n.index in visited:
                return True
            visited.add(n.index)
            if not fcond(groups[n.index].find_root().pattern, n is sink):
                return False
            if n is sink:
                return True
            return all(rec(c) for c, _ in n.outputs)
        return all(rec(c) for c, _ in src.outputs)

    def merge(child, parent):
        child, parent = child.find_root(), parent.find_root()
        if child is parent:
            return
        parent.num_nodes += child.num_nodes
        child.parent = parent
        if child.anchor is not None:
            assert parent.anchor is None, "two anchors in one group"
            parent.anchor = child.anchor
            parent.pattern = _combine(child.pattern, parent.pattern)

    def commit(src, sink):
        target = groups[sink.index]
        visited = set()

        def rec(n):
            if n is sink or n.index in visited:
                return
            visited.add(n.index)
            merge(groups[n.index], target)
            for c, _ in n.outputs:
                rec(c)
        rec(src)

    def count_with_child(child, dom_parent):
        visited = set()

        def rec(n):
            if n is dom_parent or n.index in visited:
                return 0
            visited.add(n.index)
            return groups[n.index].num_nodes + sum(rec(c) for c, _ in n.outputs)
        return groups[dom_parent.index].find_root().num_nodes + rec(child)

    def sink_ok(kind, is_sink):
        if not is_sink:
            return kind <= kInjective
        return kind <= kBroadcast or kind in (kCommReduce, kInjective, kOutEWiseFusable)

    for phase in range(3):
        for nid, gnode in enumerate(order):
            dom = tree[nid]
            grp = groups[nid]
            if grp.pattern == kOpaque or dom.parent is None:
                continue
            parent_node = dom.parent.gnode
            if count_with_child(gnode, parent_node) > max_depth:
                continue
            if phase == 2:
                continue  # tuple fusion: no tuples in these graphs
            if grp.find_root() is groups[parent_node.index].find_root():
                continue
            if groups[parent_node.index].pattern == kTuple:
                continue
            if grp.pattern == kOutEWiseFusable:
                if phase != 0:
                    continue
                if dom.pattern == kElemWise and check_path(gnode, parent_node, lambda k, s: k <= kBroadcast):
                    commit(gnode, parent_node)
            elif grp.pattern <= kBroadcast:
                if (dom.pattern <= kInjective or dom.pattern == kCommReduce) and \
                        check_path(gnode, parent_node, sink_ok):
                    commit(gnode, parent_node)
            elif grp.pattern in (kInjective, kTuple):
                if phase != 1:
                    continue
                if check_path(gnode, parent_node, lambda k, s: k <= kInjective):
                    commit(gnode, parent_node)
    return {n.name: groups[n.index].find_root() for n in order}


# ---------------------------------------------------------------- naming

_MASK = (1 << 64) - 1


def std_hash(s: str) -> int:
    """``std::hash<std::string>`` of libstdc++ on 64-bit Linux (``_Hash_bytes``, seed
    0xc70f6907): what te_compiler_cache.cc:234 appends to truncated names."""
    data = s.encode()
    mul = (0xC6A4A793 << 32) + 0x5BD1E995

    def shift_mix(v):
        return v ^ (v >> 47)
    n = len(data)
    h = (0xC70F6907 ^ (n * mul)) & _MASK
    aligned = n & ~7
    for i in range(0, aligned, 8):
        d = int.from_bytes(data[i:i + 8], "little")
        d = (shift_mix((d * mul) & _MASK) * mul) & _MASK
        h = ((h ^ d) * mul) & _MASK
    if n & 7:
        d = int.from_bytes(data[aligned:], "little")
        h = ((h ^ d) * mul) & _MASK
    h = (shift_mix(h) * mul) & _MASK
    return shift_mix(h)


def candidate_name(op_names: List[str]) -> str:
    """LowerToTECompute::Lower naming (te_compiler_cache.cc:222-236)."""
    name = "fused" + "".join("_" + n for n in op_names)
    if len(name) > MAX_FUNC_NAME_LENGTH:
        name = f"{name[:MAX_FUNC_NAME_LENGTH]}_{std_hash(name):x}_"
    return name


class NameSupply:
    """name_supply.cc:46-91."""

    def __init__(self, prefix: str = ""):
        self.prefix = prefix
        self.names: Dict[str, int] = {}

    def fresh(self, name: str, add_prefix: bool = True) -> str:
        if add_prefix and self.prefix:
            name = f"{self.prefix}_{name}"
        name = name.replace(".", "_")
        if name in self.names:
            base = name
            new = name
            while new in self.names:
                self.names[base] += 1
                new = f"{base}_{self.names[base]}"
            self.names[new] = 0
            return new
        self.names[name] = 0
        return name


@dataclass
class FusedNode:
    """One fused primitive function call of the executor graph."""
    ops: List[object]       # plan ops of the group, post order within the function body
    func_name: str          # lowered function (shared by structurally equal groups)
    node_name: str          # graph node name (FreshName(func_name))
    inputs: List[str]       # external inputs (plan tensor names), in argument order

    @property
    def output(self) -> str:
        return self.ops[-1].name


def _signature(ops, inputs, shapes) -> str:
    """Structural identity of a fused function (the TE compiler cache key): op sequence,
    attributes, folded constants and argument types."""
    h = hashlib.sha256()
    local = {x: f"arg{i}" for i, x in enumerate(inputs)}
    for k, op in enumerate(ops):
        local[op.name] = f"t{k}"
    for op in ops:
        attrs = {k: v for k, v in op.attrs.items()}
        h.update(json.dumps([op.op, [local[x] for x in op.inputs], list(op.out.shape), op.out.dtype],
                            default=str).encode())
        h.update(json.dumps(attrs, sort_keys=True, default=lambda v: np.asarray(v).tolist()).encode())
        for k in sorted(op.consts):
            h.update(k.encode() + np.ascontiguousarray(op.consts[k]).tobytes())
    for x in inputs:
        h.update(json.dumps(shapes[x]).encode())
    return h.hexdigest()


def fused_nodes(plan, mod_name: str = "default", opt_level: int = 3,
                max_depth: int = MAX_FUSED_OPS) -> List[FusedNode]:
    """The executor graph's op nodes in the order the graph codegen emits them (post order
    of the fused calls), each with its ops, function name and node name."""
    roots = partition(plan, opt_level, max_depth)
    by_name = {op.name: op for op in plan.ops}
    members: Dict[int, List[object]] = {}
    for op in plan.ops:
        members.setdefault(id(roots[op.name]), []).append(op)
    shapes = {t.name: (list(t.shape), t.dtype) for t in list(plan.inputs) + list(plan.params)}
    for op in plan.ops:
        shapes[op.name] = (list(op.out.shape), op.out.dtype)

    def group_of(name):
        return id(roots[name]) if name in by_name else None

    consumers: Dict[str, List[str]] = {}
    for op in plan.ops:
        for x in op.inputs:
            consumers.setdefault(x, []).append(op.name)

    # the fused function body, visited from its output in post order (args in order)
    def body_order(gid):
        ops = members[gid]
        sink = [o for o in ops if not any(group_of(c) == gid for c in consumers.get(o.name, []))]
        out, seen, ext = [], set(), []

        def visit(op):
            if op.name in seen:
                return
            seen.add(op.name)
            for x in op.inputs:
                if group_of(x) == gid:
                    visit(by_name[x])
                elif x not in ext:
                    ext.append(x)
            out.append(op)
        for s in sink:
            visit(s)
        return out, ext

    # the graph codegen's visit of main: post order over fused calls from the output
    order: List[int] = []
    seen_g = set()

    def visit_group(gid):
        if gid in seen_g:
            return
        seen_g.add(gid)
        _, ext = body_order(gid)
        for x in ext:
            if group_of(x) is not None:
                visit_group(group_of(x))
        order.append(gid)
    for o in plan.outputs:
        visit_group(group_of(o))
    for op in plan.ops:  # unreachable groups (none in a well-formed plan)
        visit_group(group_of(op.name))

    funcs = NameSupply(f"tvmgen_{mod_name}")
    nodes_ns = NameSupply("")
    cache: Dict[str, str] = {}
    out: List[FusedNode] = []
    for gid in order:
        ops, ext = body_order(gid)
        sig = _signature(ops, ext, shapes)
        if sig not in cache:
            cache[sig] = funcs.fresh(candidate_name([relay_op_name(o) for o in ops]))
        fn = cache[sig]
        out.append(FusedNode(ops, fn, nodes_ns.fresh(fn), ext))
    return out

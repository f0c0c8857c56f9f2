"""``relay.quantize.partition_conversions`` (python/tvm/relay/quantize/_partition_conversions.py:28-
360): split a quantized module into input quantization, the core quantized network and output
dequantization.

The result holds four functions, as in the reference: ``quantize_inputs`` (the conversion ops that
take each graph input into the quantized space; returns the tuple of converted inputs, inputs that
need no conversion passed through), ``quantized_main`` (everything between; one parameter per
converted input), ``dequantize_outputs`` (the conversion ops after the last quantized-dtype value;
parameter ``input``) and ``main``, the three composed.  The reference's ``main`` binds the three
calls with ``let``; this IR has no ``let`` or global calls, so ``main`` is the composition with
every partition's body substituted into the next -- the same computation, and the function
``relay.build`` traces.  ``ensure_fully_integral`` (``partition_conversions="fully_integral"``)
raises AssertionError when the prefix or suffix holds other than conversion ops or the core holds
other than the quantized dtypes, like the reference's assertions (:79-83).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Set

from ..expr import Call, Constant, Expr, Function, IRModule, Tuple, Var, free_vars, post_order

# operators allowed in the prefix / suffix partitions (_partition_conversions.py:25)
ALLOWED_CONVERSION_OPS = ["add", "multiply", "right_shift", "clip", "round", "cast"]


def _substitute(body: Expr, mapping: Dict[int, Expr]) -> Expr:
    """``body`` with every Var whose id is in ``mapping`` replaced (post-order rebuild)."""
    new: Dict[int, Expr] = dict(mapping)
    for n in post_order(body):
        if isinstance(n, Call):
            args = [new.get(id(x), x) for x in n.args]
            if any(x is not y for x, y in zip(args, n.args)):
                new[id(n)] = Call(n.op, args, n.attrs, n.checked_type)
        elif isinstance(n, Tuple):
            fields = [new.get(id(x), x) for x in n.fields]
            if any(x is not y for x, y in zip(fields, n.fields)):
                new[id(n)] = Tuple(fields)
    return new.get(id(body), body)


class _PrefixCutter:
    """PrefixCutter (_partition_conversions.py:137-172): above the first non-conversion op on each
    path, a subtree that reads exactly one graph parameter is cut out as that parameter's input
    conversion and replaced by a new parameter of the core function."""

    def __init__(self, params: List[Var]):
        self.params = {id(p) for p in params}
        self.subtree_params: List[Var] = []
        self.memo: Dict[int, Expr] = {}
        self.bindings: Dict[int, Expr] = {}   # id(mid param) -> its prefix expression
        self.mid_params: Dict[int, Var] = {}

    def visit(self, e: Expr) -> Expr:
        if id(e) in self.memo:
            return self.memo[id(e)]
        if isinstance(e, Var):
            if id(e) in self.params and all(p is not e for p in self.subtree_params):
                self.subtree_params.append(e)
            out = e
        elif isinstance(e, Call) and e.op not in ALLOWED_CONVERSION_OPS:
            new_args = []
            for arg in e.args:
                na = self.visit(arg)
                if not self.subtree_params:
                    new_args.append(na)
                    continue
                assert len(self.subtree_params) == 1, "a conversion subtree reads more than one input"
                param = self.subtree_params.pop()
                mid = Var(param.name_hint, arg.shape, arg.dtype)
                self.bindings[id(mid)] = na
                self.mid_params[id(mid)] = mid
                new_args.append(mid)
            out = Call(e.op, new_args, e.attrs, e.checked_type)
        elif isinstance(e, Call):
            args = [self.visit(a) for a in e.args]
            out = e if all(x is y for x, y in zip(args, e.args)) else Call(e.op, args, e.attrs, e.checked_type)
        elif isinstance(e, Tuple):
            fields = [self.visit(f) for f in e.fields]
            out = e if all(x is y for x, y in zip(fields, e.fields)) else Tuple(fields)
        else:
            out = e
        self.memo[id(e)] = out
        return out


def partition_prefix(mod: IRModule):
    """(pre_mod, mid_mod): the input quantization and everything after it (:175-226)."""
    func = mod["main"]
    cutter = _PrefixCutter(func.params)
    mid_body = cutter.visit(func.body)
    mid_params = free_vars(mid_body)
    rets: List[Expr] = []
    for p in mid_params:
        # a converted input: its conversion; another input: passed through
        rets.append(cutter.bindings.get(id(p), p))
    pre_body = Tuple(rets)
    pre_func = Function(free_vars(pre_body), pre_body)
    return IRModule(pre_func), IRModule(Function(mid_params, mid_body)), cutter.bindings


class _SuffixCutter:
    """SuffixCutter (:229-245): top-down, the first value of a quantized dtype on each path is
    the core's result; it becomes the suffix function's parameter ``input``."""

    def __init__(self, quantized_dtypes: Set[str]):
        self.qd = quantized_dtypes
        self.mid_body: Optional[Expr] = None
        self.input: Optional[Var] = None
        self.memo: Dict[int, Expr] = {}

    def visit(self, e: Expr) -> Expr:
        if id(e) in self.memo:
            return self.memo[id(e)]
        if not isinstance(e, Tuple) and e.dtype in self.qd:
            self.mid_body = e
            if self.input is None or self.input.shape != e.shape or self.input.dtype != e.dtype:
                self.input = Var("input", e.shape, e.dtype)
            out = self.input
        elif isinstance(e, Call):
            args = [self.visit(a) for a in e.args]
            out = e if all(x is y for x, y in zip(args, e.args)) else Call(e.op, args, e.attrs, e.checked_type)
        elif isinstance(e, Tuple):
            out = Tuple([self.visit(f) for f in e.fields])
        else:
            out = e
        self.memo[id(e)] = out
        return out


def partition_suffix(mod: IRModule, quantized_dtypes: Set[str]):
    """(mid_mod, post_mod): the core and the output dequantization (:248-290)."""
    func = mod["main"]
    cutter = _SuffixCutter(quantized_dtypes)
    post_body = cutter.visit(func.body)
    if cutter.mid_body is None:
        # no quantization boundary: the whole function is the core, the suffix the identity
        ident = Var("input", func.body.shape, func.body.dtype)
        return IRModule(func), IRModule(Function([ident], ident)), None
    post_func = Function(free_vars(post_body), post_body)
    return IRModule(Function(func.params, cutter.mid_body)), IRModule(post_func), cutter.input


def _only_conversion_ops(func: Function) -> bool:
    """has_only_conversion_ops (:293-345)."""
    return all(n.op in ALLOWED_CONVERSION_OPS for n in post_order(func.body) if isinstance(n, Call))


def _all_dtypes(func: Function) -> Set[str]:
    """relay.analysis.all_dtypes: the dtypes of every parameter, constant and call."""
    out = {p.dtype for p in func.params}
    for n in post_order(func.body):
        if isinstance(n, (Call, Var, Constant)):
            out.add(n.dtype)
    return out


def partition_conversions(mod: IRModule, quantized_dtypes: Set[str], ensure_fully_integral: bool) -> IRModule:
    """The quantize_inputs / quantized_main / dequantize_outputs / main module (:28-84)."""
    if len(mod.functions) != 1:
        raise ValueError("partition_conversions: a module with one function expected")
    pre_mod, mid_mod, bindings = partition_prefix(mod)
    mid_mod, post_mod, post_input = partition_suffix(mid_mod, set(quantized_dtypes))
    if ensure_fully_integral:
        assert _only_conversion_ops(pre_mod["main"]), "the input quantization holds other than conversion ops"
        assert _all_dtypes(mid_mod["main"]).issubset(set(quantized_dtypes)), \
            "the core holds other than quantized dtypes"
        assert _only_conversion_ops(post_mod["main"]), "the output dequantization holds other than conversion ops"
    pre, mid, post = pre_mod["main"], mid_mod["main"], post_mod["main"]
    # main = dequantize_outputs(quantized_main(*quantize_inputs(*params))), composed by substitution
    mid_in = {id(p): bindings.get(id(p), p) for p in mid.params}
    core = _substitute(mid.body, mid_in)
    body = _substitute(post.body, {id(post.params[0]): core}) if post_input is not None else core
    main = Function(list(mod["main"].params), body)
    return IRModule(main, {"quantize_inputs": pre, "quantized_main": mid, "dequantize_outputs": post})

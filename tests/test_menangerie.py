"""The reference's own float test models as Relay text (tests/golden/menangerie_*.relay, extracted
from tests/python/relay/collage/menangerie.py by tools/extract_menangerie.py): parsing
(``nn.batch_norm`` and its ``%k.0`` field, ``nn.pad`` with the pad value as an argument, ``reshape``
with 0 / -1), the SimplifyInference / FoldScaleAxis prerequisites of ``relay.quantize``
(quantize.py:312-322) and quantization of the parsed models.  The device traces of the quantized
models are tests/test_gpu_ingest.py."""
import re

import numpy as np
import pytest

from oracle import graph_ref
from tachikoma_amd import relay
from tachikoma_amd.relay import transform
from tachikoma_amd.relay.quantize import passes, qconfig, quantize

from .golden_util import HERE, menangerie

MODELS = ["mnist", "resnet50", "mobilenet"]


def _ops(mod):
    return [n.op for n in relay.post_order(mod["main"].body) if isinstance(n, relay.Call)]


@pytest.mark.parametrize("name", MODELS)
def test_menangerie_parses(name):
    with open(f"{HERE}/golden/menangerie_{name}.relay") as f:
        text = f.read()
    mod, iname, shape = menangerie(name)
    ops = _ops(mod)
    # every `= op(` line of the text is one call (field projections `%k.0` are not)
    want = re.findall(r"(?:=\s*|^\s*)([a-z_][a-z0-9_.]*)\(", text, re.M)
    assert sorted(ops) == sorted(w for w in want if w != "def")
    assert mod["main"].params[0].name_hint == iname and mod["main"].params[0].shape == shape
    assert mod["main"].body.shape[-1] == 10 if name == "mnist" else mod["main"].body.shape == (1, 1000)
    # the printer writes batch norms as a tuple plus its field-0 projection; the text re-parses
    again = relay.parse(mod.astext())
    assert _ops(again) == ops
    x = np.random.default_rng(1).standard_normal(shape).astype(np.float32)
    s1 = graph_ref.calibrate(transform.fold_constant(transform.simplify_inference(mod)), {}, {iname: x})
    s2 = graph_ref.calibrate(transform.fold_constant(transform.simplify_inference(again)), {}, {iname: x})
    assert np.array_equal(list(s1.values())[-1], list(s2.values())[-1])


def test_tuple_field_errors():
    src = '''def @main(%x: Tensor[(1, 2, 2, 2), float32]) {
      %0 = nn.batch_norm(%x, meta[relay.Constant][0], meta[relay.Constant][0], meta[relay.Constant][0],
                         meta[relay.Constant][0]);
      %1 = %0.1;
      %1
    }'''
    meta = {"relay.Constant": [np.ones(2, np.float32)]}
    with pytest.raises(relay.ParseError):
        relay.parse(src, init_meta_table=meta)
    with pytest.raises(relay.ParseError):
        relay.parse(src.replace("%0.1", "nn.relu(%0)"), init_meta_table=meta)


def test_simplify_inference_is_the_reference_arithmetic():
    """BatchNormToInferUnpack (simplify_inference.cc:33-62) + FoldConstant: the scale and shift are
    float32 constants computed op by op, the output is x * scale + shift (two roundings)."""
    rng = np.random.default_rng(3)
    c = 6
    x = relay.var("x", (2, c, 5, 5))
    g, b, m, v = (rng.uniform(0.5, 1.5, c).astype(np.float32), rng.uniform(-1, 1, c).astype(np.float32),
                  rng.uniform(-1, 1, c).astype(np.float32), rng.uniform(0.1, 2.0, c).astype(np.float32))
    bn = relay.nn.batch_norm(x, *[relay.const(a) for a in (g, b, m, v)], epsilon=2e-5)[0]
    mod = relay.IRModule.from_expr(relay.nn.relu(bn))
    simp = transform.fold_constant(transform.simplify_inference(mod))
    assert _ops(simp) == ["multiply", "add", "nn.relu"]
    f32 = np.float32
    scale = (f32(1.0) / np.sqrt(v + f32(2e-5))).astype(f32) * g
    shift = (-m * scale).astype(f32) + b
    xv = rng.standard_normal((2, c, 5, 5)).astype(f32)
    exp = np.maximum((xv * scale[:, None, None]).astype(f32) + shift[:, None, None], f32(0))
    got = list(graph_ref.calibrate(simp, {}, {"x": xv}).values())[-1]
    assert got.dtype == np.float32 and np.array_equal(got, exp)


def _conv(x, o, k=1, seed=0):
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal((o, x.shape[1], k, k)) * 0.2).astype(np.float32)
    return relay.nn.conv2d(x, relay.const(w), padding=(k // 2,) * 4)


def _bn(x, seed=0):
    rng = np.random.default_rng(100 + seed)
    c = x.shape[1]
    vals = [rng.uniform(0.5, 1.5, c), rng.uniform(-0.2, 0.2, c), rng.uniform(-0.2, 0.2, c), rng.uniform(0.5, 1.5, c)]
    return relay.nn.batch_norm(x, *[relay.const(v.astype(np.float32)) for v in vals])[0]


def test_fold_scale_axis_backward():
    """A batch norm right after a conv, or after an add of two single-use convs, folds into the
    weights (no multiply left); one after an add whose operand has another consumer stays."""
    x = relay.var("x", (1, 8, 6, 6))
    a = _conv(x, 16, 1, 0)
    b = _conv(x, 16, 3, 1)
    s = relay.add(a, b)
    y = relay.nn.relu(_bn(_conv(x, 16, 3, 2), 0))     # conv -> bn: folds
    z = relay.nn.relu(_bn(s, 1))                        # add(conv, conv) -> bn: folds into both
    t = relay.add(_conv(y, 16, 1, 3), z)
    u = relay.nn.relu(_bn(t, 2))                        # t is also read below: stays
    out = relay.add(u, t)
    mod = relay.IRModule.from_expr(out)
    pre = passes.prerequisite_optimize(mod)
    ops = _ops(pre)
    assert ops.count("multiply") == 1 and ops.count("nn.batch_norm") == 0
    xv = np.random.default_rng(5).standard_normal((1, 8, 6, 6)).astype(np.float32)
    ref = list(graph_ref.calibrate(transform.fold_constant(transform.simplify_inference(mod)), {},
                                   {"x": xv}).values())[-1]
    got = list(graph_ref.calibrate(pre, {}, {"x": xv}).values())[-1]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)


def test_fold_scale_axis_add_constant_must_broadcast_on_channels():
    """add(conv, b) * s[c] with b of shape (W,) on an NCHW output where W == C: b broadcasts along
    W, not along channels, so the multiply must stay (MatchBroadcastToLeftAxes); b of shape
    (C, 1, 1) folds."""
    c = 6
    x = relay.var("x", (1, 4, c, c))
    rng = np.random.default_rng(7)
    s = relay.const(rng.uniform(0.5, 1.5, (c, 1, 1)).astype(np.float32))
    xv = rng.standard_normal((1, 4, c, c)).astype(np.float32)
    for bshape, folds in (((c,), False), ((c, 1, 1), True), ((1, c, 1, 1), True)):
        b = relay.const(rng.uniform(-1, 1, bshape).astype(np.float32))
        mod = relay.IRModule.from_expr(relay.multiply(relay.add(_conv(x, c, 3, 4), b), s))
        out = transform.fold_constant(transform.fold_scale_axis(mod))
        assert ("multiply" not in _ops(out)) == folds, bshape
        ref = list(graph_ref.calibrate(transform.fold_constant(mod), {}, {"x": xv}).values())[-1]
        got = list(graph_ref.calibrate(out, {}, {"x": xv}).values())[-1]
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("groups,depthwise", [(1, False), (2, False), (8, True)])
def test_fold_scale_axis_grouped_conv(groups, depthwise):
    """ConvBackwardPrep folds only into groups == 1 or depthwise convs (fold_scale_axis.cc:986-987)."""
    rng = np.random.default_rng(11)
    x = relay.var("x", (1, 8, 5, 5))
    w = rng.standard_normal((8, 8 // groups, 3, 3)).astype(np.float32)
    conv = relay.nn.conv2d(x, relay.const(w), padding=(1, 1, 1, 1), groups=groups)
    s = relay.const(rng.uniform(0.5, 1.5, (8, 1, 1)).astype(np.float32))
    mod = relay.IRModule.from_expr(relay.multiply(conv, s))
    out = transform.fold_constant(transform.fold_scale_axis(mod))
    assert ("multiply" not in _ops(out)) == (groups == 1 or depthwise)
    xv = rng.standard_normal((1, 8, 5, 5)).astype(np.float32)
    ref = list(graph_ref.calibrate(transform.fold_constant(mod), {}, {"x": xv}).values())[-1]
    got = list(graph_ref.calibrate(out, {}, {"x": xv}).values())[-1]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", ["mnist", "mobilenet"])
def test_quantize_menangerie(name):
    """relay.quantize of a parsed reference model: every batch norm of a conv -> bn chain is
    folded into the conv weights before annotation, the integer graph runs on the oracle."""
    mod, iname, shape = menangerie(name)
    with qconfig(skip_conv_layers=[0]):
        q = quantize(mod, {})
    ops = _ops(q)
    assert "nn.batch_norm" not in ops and "relay.op.annotation.simulated_quantize" not in ops
    convs = [n for n in relay.post_order(q["main"].body) if isinstance(n, relay.Call) and n.op == "nn.conv2d"]
    # all but the skipped first one and, in mobilenet, the classifier conv after the global pool
    # (global_avg_pool2d stops quantization, _annotate.py:395-409)
    assert sum(c.args[0].dtype == "int8" for c in convs) == len(convs) - (2 if name == "mobilenet" else 1)
    if name == "mobilenet":
        assert ops.count("multiply") <= 2  # the input quantize and the output dequantize
    x = np.random.default_rng(2).standard_normal(shape).astype(np.float32)
    rec = graph_ref.calibrate(q, {}, {iname: x})
    out = list(rec.values())[-1]
    assert out.shape[-1] in (10, 1000) and np.isfinite(out).all()

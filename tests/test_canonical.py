"""The canonical graph behind the fused-node debug dump (tachikoma_amd/relay/canonical.py):
fused-function names against the reference's own quantized-model structures
(tests/python/unittest/test_tir_usmp_algo.py:295-520), the SimplifyExpr rewrites, and the
canonical values against the QNN oracle records they equal (oracle/canonical_ref.py)."""
import numpy as np
import pytest

from oracle import canonical_ref, graph_ref
from tachikoma_amd import relay, zoo
from tachikoma_amd.relay import qnn
from tachikoma_amd.relay.build_module import lower
from tachikoma_amd.relay.canonical import canonicalize
from tachikoma_amd.relay.fuse import fused_nodes


def _c(v, dt):
    return relay.const(v, dt)


def _conv(x, name, cin, cout, k, zp_in, params, rng, stride=1, pad=0, zp_out=0, s_ratio=0.003, out="uint8"):
    w = relay.var(f"{name}.w", (cout, cin, k, k), "int8")
    b = relay.var(f"{name}.b", (cout,), "int32")
    params[f"{name}.w"] = rng.integers(-128, 128, (cout, cin, k, k)).astype(np.int8)
    params[f"{name}.b"] = rng.integers(-1000, 1000, cout).astype(np.int32)
    y = qnn.op.conv2d(x, w, _c(zp_in, "int32"), _c(0, "int32"), _c(0.05, "float32"), _c(0.01, "float32"),
                      kernel_size=(k, k), channels=cout, strides=(stride, stride), padding=pad)
    y = relay.nn.bias_add(y, b, axis=1)
    return qnn.op.requantize(y, _c(np.float32(0.05 * 0.01), "float32"), _c(0, "int32"),
                             _c(np.float32(0.05 * 0.01 / s_ratio), "float32"), _c(zp_out, "int32"), axis=1,
                             out_dtype=out)


def _names(mod, params, **kw):
    return [n.func_name for n in fused_nodes(canonicalize(lower(mod, params), **kw))]


def test_mobilenet_structure_names():
    """test_tir_usmp_algo.py:297-361 (MobilenetStructure): a uint8 input with a non-zero zero point,
    the 7x7/2 stem conv block (per-tensor requantize to uint8, zero points 0), a 3x3/2 max pool
    feeding the next conv: fused_cast_subtract, fused_nn_conv2d_add_fixed_point_multiply_clip_cast,
    fused_nn_max_pool2d_cast."""
    rng = np.random.default_rng(0)
    params = {}
    x = relay.var("input", (1, 3, 224, 224), "uint8")
    y = _conv(x, "stem", 3, 64, 7, 128, params, rng, stride=2, pad=(2, 2, 3, 3))
    y = relay.nn.max_pool2d(y, pool_size=(3, 3), strides=(2, 2), padding=(0, 0, 1, 1))
    y = _conv(y, "next", 64, 64, 1, 0, params, rng)
    names = _names(relay.IRModule.from_expr(y), params)
    assert names[:3] == ["tvmgen_default_fused_cast_subtract",
                         "tvmgen_default_fused_nn_conv2d_add_fixed_point_multiply_clip_cast",
                         "tvmgen_default_fused_nn_max_pool2d_cast"]


def _resnet_structure():
    """ResnetStructure (test_tir_usmp_algo.py:418-520): a requantize of the uint8 input (zero point
    94), a 1x1 and a 3x3 conv block, then the bottleneck's 1x1 expand and the 1x1 downsample joined
    by qnn.add (output zero points 132 / 136)."""
    rng = np.random.default_rng(1)
    params = {}
    x = relay.var("input", (1, 64, 75, 75), "uint8")
    r = qnn.op.requantize(x, _c(0.02, "float32"), _c(94, "int32"), _c(0.011, "float32"), _c(3, "int32"),
                          out_dtype="uint8")
    a = _conv(r, "c1", 64, 64, 1, 0, params, rng)
    a = _conv(a, "c2", 64, 64, 3, 0, params, rng, pad=1)
    e = _conv(a, "c3", 64, 256, 1, 0, params, rng, zp_out=132)
    d = _conv(r, "ds", 64, 256, 1, 0, params, rng, zp_out=136)
    y = qnn.op.add(e, d, _c(0.05, "float32"), _c(132, "int32"), _c(0.06, "float32"), _c(136, "int32"),
                   _c(0.07, "float32"), _c(136, "int32"))
    return relay.IRModule.from_expr(y), params


def test_resnet_structure_names():
    """The requantize-of-the-input group and the conv groups whose output is the next conv's int16
    operand (clip -> cast uint8 -> cast int16 survives SimplifyExpr: the second cast is not back
    to the clip's int32) carry the reference's names; a structurally different function with the
    same name gets NameSupply's _1 (name_supply.cc:46-91)."""
    mod, params = _resnet_structure()
    names = _names(mod, params)
    assert names[0] == "tvmgen_default_fused_cast_subtract_fixed_point_multiply_add_clip_cast_cast"
    assert "tvmgen_default_fused_nn_conv2d_add_fixed_point_multiply_clip_cast_cast" in names
    assert "tvmgen_default_fused_nn_conv2d_add_fixed_point_multiply_clip_cast_cast_1" in names
    # the qnn.add tails are longer than kMaxFuncNameLength: 80 characters, then std::hash in hex
    long = [n for n in names if len(n) > len("tvmgen_default_") + 80]
    assert long and all(n.endswith("_") and int(n[len("tvmgen_default_") + 81:-1].split("_")[0], 16) >= 0
                        for n in long)


def test_resnet_structure_add_groups_without_clip_cast_simplification():
    """The usmp fixture's qnn.add groups read ``cast(cast(clip(..), uint8), int32)``, which the
    reference's SimplifyClipAndConsecutiveCast (simplify_expr.cc:183-235, registered at :967)
    reduces to the clip -- and they end in a *decimal* hash where te_compiler_cache.cc:234 prints
    hex: that TIR predates the reference's source.  With the rewrite off, the 80-character prefix
    is the fixture's."""
    mod, params = _resnet_structure()
    names = _names(mod, params, simplify_clip_cast=False)
    prefix = "tvmgen_default_fused_nn_conv2d_add_fixed_point_multiply_add_clip_cast_cast_subtract_fixed_point"
    assert sum(n.startswith(prefix + "_") for n in names) == 2
    on = _names(mod, params)
    assert not any(n.startswith(prefix + "_") for n in on)


@pytest.mark.parametrize("name", ["resnet18", "mobilenet_v2", "lenet5"])
def test_canonical_values_equal_their_records(name):
    """Every canonical op that stands for a plan record evaluates (oracle/canonical_ref.py) to
    exactly that record (graph_ref, the QNN oracle); every op has a fused group."""
    m = zoo.MODELS[name](batch=1)
    plan = lower(m.mod, m.params)
    canon = canonicalize(plan)
    x = m.random_input()
    vals = canonical_ref.evaluate(canon, {m.input_name: x, **{k: np.asarray(v) for k, v in m.params.items()}})
    rec = graph_ref.calibrate(m.mod, m.params, {m.input_name: x}, backend="c")
    checked = 0
    for op in canon.ops:
        if op.record is not None:
            assert np.array_equal(vals[op.name], rec[op.record]), (op.name, op.op, op.record)
            checked += 1
    assert checked >= len(plan.ops) * 0.8
    nodes = fused_nodes(canon)
    assert sum(len(n.ops) for n in nodes) == len(canon.ops)
    assert all(n.func_name.startswith("tvmgen_default_fused_") for n in nodes)


def test_tonearest_requantize_lowering():
    """TONEAREST requantize lowers like FixedPointMultiplyToNearest (src/relay/qnn/utils.cc:59-216):
    int64 cast, multiply, greater_equal / where rounding constant, add, right_shift, cast -- per
    tensor and per channel; the values still equal the plan's records and the ops fuse into the
    producer's function (its name lists them)."""
    from tachikoma_amd.relay import qnn
    with qnn.op.requantize_config(rounding="TONEAREST"):
        m = zoo.lenet5(batch=2)
    plan = lower(m.mod, m.params)
    assert all(o.attrs["rounding"] == "TONEAREST" for o in plan.ops if o.op == "qnn.requantize")
    canon = canonicalize(plan)
    kinds = [o.op for o in canon.ops]
    assert "fixed_point_multiply" not in kinds and "fixed_point_multiply_per_axis" not in kinds
    assert {"greater_equal", "where", "right_shift", "multiply"} <= set(kinds)
    x = m.random_input()
    vals = canonical_ref.evaluate(canon, {m.input_name: x, **{k: np.asarray(v) for k, v in m.params.items()}})
    rec = graph_ref.calibrate(m.mod, m.params, {m.input_name: x})
    checked = [op for op in canon.ops if op.record is not None]
    for op in checked:
        assert np.array_equal(vals[op.name], rec[op.record]), (op.name, op.op, op.record)
    assert any(r.op == "qnn.requantize" for r in plan.ops if r.name in {o.record for o in checked})
    names = [n.func_name for n in fused_nodes(canon)]
    assert any("greater_equal_where" in n for n in names), names


@pytest.mark.parametrize("rounding", ["UPWARD", "TONEAREST"])
def test_per_axis_qnn_add_lowering(rounding):
    """qnn.add with a per-axis side (scales and zero points along lhs_axis) and the rounding of the
    requantize_config it was built under: each side lowers to its own Requantize (RequantizeOrUpcast,
    src/relay/qnn/op/op_common.h:186-207) along that side's axis, and the canonical values equal the
    QNN oracle's record; a broadcasting add is refused, not lowered wrongly."""
    x = relay.var("x", (2, 3, 4, 5), "int8")
    y = relay.var("y", (2, 3, 4, 5), "int8")
    with qnn.op.requantize_config(rounding=rounding):
        e = qnn.op.add(x, y, relay.const(np.array([0.11, 0.23, 0.37], np.float32)),
                       relay.const(np.array([1, -3, 4], np.int32)), 0.25, 1, 0.5, 2, lhs_axis=1)
    mod = relay.IRModule.from_expr(e)
    plan = lower(mod, {})
    (op,) = plan.ops
    assert op.attrs["rounding"] == rounding and "lhs_multipliers" in op.consts and not op.attrs["per_tensor"]
    canon = canonicalize(plan)
    kinds = [o.op for o in canon.ops]
    if rounding == "UPWARD":
        assert "fixed_point_multiply_per_axis" in kinds
    else:
        assert "fixed_point_multiply_per_axis" not in kinds and "where" in kinds
    rng = np.random.default_rng(3)
    xs = {"x": rng.integers(-128, 128, (2, 3, 4, 5), dtype=np.int8),
          "y": rng.integers(-128, 128, (2, 3, 4, 5), dtype=np.int8)}
    vals = canonical_ref.evaluate(canon, dict(xs))
    rec = graph_ref.calibrate(mod, {}, xs)
    rop = [o for o in canon.ops if o.record is not None]
    assert rop and all(np.array_equal(vals[o.name], rec[o.record]) for o in rop)
    b = qnn.op.add(x, relay.var("z", (3, 1, 1), "int8"), 0.5, 0, 0.25, 1, 0.5, 0)
    with pytest.raises(relay.UnsupportedError if hasattr(relay, "UnsupportedError") else Exception):
        canonicalize(lower(relay.IRModule.from_expr(b), {}))

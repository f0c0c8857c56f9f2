"""Host side of the pre-quantized QNN ops, no GPU: Relay text with tuples,
lowering to plan ops (requantize plans of qnn.concatenate / mul / subtract, quantize parameters,
conv layouts), MRT naming (tuples take no %N), and the oracle's layout semantics pinned to the
reference's own property (qnn.conv2d == nn.conv2d of the shifted operands in each layout,
tests/python/relay/test_op_qnn_conv2d.py:35-82, 494-545)."""
import numpy as np
import pytest

from oracle import graph_ref
from oracle import qnn_ref as ref
from tachikoma_amd import relay
from tachikoma_amd.relay import qnn
from tachikoma_amd.relay.build_module import UnsupportedError, build, exec_groups

from .test_gpu_qnn_ops import QNN_TEXT


def _params(rng):
    return {"w": rng.integers(-128, 128, (3, 3, 16, 32)).astype(np.int8),
            "b": rng.integers(-5000, 5000, 32).astype(np.int32)}


def test_text_graph_lowers_with_mrt_names():
    mod = relay.parse(QNN_TEXT)
    assert relay.parse(mod.astext()).astext() == mod.astext()
    plan = build(mod, params=_params(np.random.default_rng(0))).plan
    assert [o.op for o in plan.ops] == ["qnn.quantize", "qnn.conv2d", "nn.bias_add", "qnn.requantize", "clip",
                                        "qnn.concatenate", "qnn.mul", "qnn.subtract", "qnn.dequantize"]
    assert [o.name for o in plan.ops] == [f"%{i}" for i in range(9)]  # the tuple takes no name
    by = {o.op: o for o in plan.ops}
    assert by["qnn.concatenate"].inputs == ["%4", "y"]
    assert by["qnn.conv2d"].out.shape == (2, 14, 14, 32) and by["qnn.concatenate"].out.shape == (2, 14, 14, 40)
    # concatenate: both inputs' params differ from the output's -> requantized to it
    assert [p["requant"] for p in by["qnn.concatenate"].attrs["inputs"]] == [1, 1]
    assert by["qnn.quantize"].attrs["scale"] == float(np.float32(0.05)) and by["qnn.quantize"].attrs["axis"] == 3
    # the NHWC conv is not fused into a block (the block kernels are NCHW); everything is traced
    kinds = [g.kind for g in exec_groups(plan)]
    assert "conv_block" not in kinds and len(kinds) == 9


def test_text_graph_oracle_runs():
    mod = relay.parse(QNN_TEXT)
    rng = np.random.default_rng(1)
    params = _params(rng)
    x = rng.standard_normal((1, 14, 14, 16)).astype(np.float32)
    y = rng.integers(-128, 128, (1, 14, 14, 8)).astype(np.int8)
    rec = graph_ref.calibrate(mod, params, {"x": x, "y": y})
    assert set(rec) == {"x", "y"} | {f"%{i}" for i in range(9)}
    assert rec["%8"].dtype == np.float32 and rec["%5"].shape == (1, 14, 14, 40)
    # the concatenation is the two requantized inputs side by side on axis 3
    a = ref.requantize(rec["%4"], np.float32(0.1), np.int32(2), np.float32(0.09), np.int32(1), out_dtype="int8")
    b = ref.requantize(y, np.float32(0.07), np.int32(-1), np.float32(0.09), np.int32(1), out_dtype="int8")
    np.testing.assert_array_equal(rec["%5"], np.concatenate([a, b], axis=3))


def _conv_nhwc_direct(x, w_hwio, za, zw, pad):
    """nn.conv2d(cast(x) - za, cast(w) - zw) written directly in NHWC / HWIO (no transposes)."""
    n, h, wd, c = x.shape
    kh, kw, ci, o = w_hwio.shape
    xs = np.pad(x.astype(np.int64) - za, ((0, 0), (pad, pad), (pad, pad), (0, 0)))
    ws = w_hwio.astype(np.int64) - zw
    oh, ow = h + 2 * pad - kh + 1, wd + 2 * pad - kw + 1
    out = np.zeros((n, oh, ow, o), np.int64)
    for r in range(kh):
        for s in range(kw):
            out += np.einsum("nhwc,co->nhwo", xs[:, r:r + oh, s:s + ow, :], ws[r, s])
    return ref.wrap_i32(out).astype(np.int32)


@pytest.mark.parametrize("kernel_layout", ["HWIO", "OHWI", "HWOI", "OIHW"])
def test_oracle_conv_layouts_equal_direct_nhwc(kernel_layout):
    rng = np.random.default_rng(2)
    x = rng.integers(0, 256, (2, 6, 5, 4)).astype(np.uint8)
    w_hwio = rng.integers(0, 256, (3, 3, 4, 6)).astype(np.uint8)
    w = np.ascontiguousarray(w_hwio.transpose(["HWIO".index(ch) for ch in kernel_layout]))
    vx, vw = relay.var("x", x.shape, "uint8"), relay.var("w", w.shape, "uint8")
    e = qnn.op.conv2d(vx, vw, relay.const(5, "int32"), relay.const(3, "int32"), relay.const(1.0), relay.const(1.0),
                      kernel_size=(3, 3), channels=6, padding=(1, 1), data_layout="NHWC", kernel_layout=kernel_layout)
    assert e.shape == (2, 6, 5, 6)
    got = graph_ref.calibrate(relay.IRModule.from_expr(e), {"w": w}, {"x": x})["%0"]
    np.testing.assert_array_equal(got, _conv_nhwc_direct(x, w_hwio, 5, 3, 1))


def test_depthwise_multiplier_form():
    """(C, M, KH, KW) depthwise weights (Conv2DRel, convolution.cc:243-274): output channel c * M + m
    reads weight[c, m] (topi depthwise_conv2d_nchw), kernel zero points along C."""
    rng = np.random.default_rng(4)
    x = rng.integers(-128, 128, (1, 4, 6, 6)).astype(np.int8)
    w = rng.integers(-128, 128, (4, 2, 3, 3)).astype(np.int8)
    zw = np.array([1, -2, 3, 0], np.int32)
    vx, vw = relay.var("x", x.shape, "int8"), relay.var("w", w.shape, "int8")
    e = qnn.op.conv2d(vx, vw, relay.const(-3, "int32"), relay.const(zw), relay.const(1.0), relay.const(1.0),
                      kernel_size=(3, 3), channels=8, groups=4)
    assert e.shape == (1, 8, 4, 4) and e.attrs["depthwise_multiplier"] == 2
    got = graph_ref.calibrate(relay.IRModule.from_expr(e), {"w": w}, {"x": x})["%0"]
    exp = np.zeros((1, 8, 4, 4), np.int64)
    for c in range(4):
        for m in range(2):
            for r in range(3):
                for s in range(3):
                    exp[0, c * 2 + m] += (x[0, c, r:r + 4, s:s + 4].astype(np.int64) + 3) * (int(w[c, m, r, s]) - zw[c])
    np.testing.assert_array_equal(got, exp.astype(np.int32))
    plan = build(relay.IRModule.from_expr(e), params={"w": w}).plan
    assert plan.ops[0].consts["kernel_zero_points"].tolist() == [1, 1, -2, -2, 3, 3, 0, 0]
    with pytest.raises(TypeError):
        qnn.op.conv2d(vx, vw, relay.const(0, "int32"), relay.const(0, "int32"), relay.const(1.0), relay.const(1.0),
                      kernel_size=(3, 3), channels=6, groups=4)


def test_lowering_plans():
    x = relay.var("x", (2, 3, 4, 5), "int8")
    y = relay.var("y", (3, 1, 1), "int8")
    sub = qnn.op.subtract(x, y, 0.5, 0, 0.5, 0, 0.5, 0)
    add = qnn.op.add(x, x, 0.5, 0, 0.25, 1, 0.5, 0)
    mul = qnn.op.mul(x, x, relay.const(np.array([0.1, 0.2, 0.3], np.float32)), 0,
                     relay.const(np.array([0.5, 0.5, 0.25], np.float32)), 1, 0.2, 0, lhs_axis=1, rhs_axis=1)
    plan = build(relay.IRModule.from_expr(mul)).plan
    op = plan.ops[0]
    assert op.attrs["out_mode"] >= 4 and len(op.consts["out_multipliers"]) == 3  # per-axis requantize
    plan = build(relay.IRModule.from_expr(sub)).plan
    o = plan.ops[0].attrs
    assert o["lhs_upcast"] == o["rhs_upcast"] == 1 and not o["per_tensor"]  # broadcast: the general kernel
    plan = build(relay.IRModule.from_expr(add)).plan
    o = plan.ops[0].attrs
    assert o["lhs_upcast"] == 1 and o["rhs_upcast"] == 0 and o["per_tensor"]
    groups = exec_groups(plan)
    assert [g.kind for g in groups] == ["add_block"]
    # unequal axes in a per-channel qnn.mul: the reference refuses them too (mul.cc:154-156)
    bad = qnn.op.mul(x, x, relay.const(np.array([0.1, 0.2, 0.3], np.float32)), 0,
                     relay.const(np.array([0.1, 0.2, 0.3, 0.4], np.float32)), 0, 0.2, 0, lhs_axis=1, rhs_axis=2)
    with pytest.raises(UnsupportedError):
        build(relay.IRModule.from_expr(bad))


def test_type_errors():
    x = relay.var("x", (2, 3), "int8")
    with pytest.raises(TypeError):
        qnn.op.quantize(x, 0.5, 0)  # quantize takes float32
    with pytest.raises(TypeError):
        qnn.op.dequantize(relay.var("f", (2, 3), "float32"), 0.5, 0)
    with pytest.raises(TypeError):
        qnn.op.concatenate((x, relay.var("z", (2, 3), "uint8")), (0.5, 0.5), (0, 0), 0.5, 0, axis=0)
    with pytest.raises(TypeError):
        qnn.op.concatenate((x, relay.var("z", (3, 3), "int8")), (0.5, 0.5), (0, 0), 0.5, 0, axis=1)
    with pytest.raises(TypeError):
        qnn.op.mul(x, relay.var("z", (4,), "int8"), 0.5, 0, 0.5, 0, 0.5, 0)  # does not broadcast
    with pytest.raises(NotImplementedError):
        qnn.op.conv2d(relay.var("d", (1, 4, 4, 3), "int8"), relay.var("k", (3, 3, 3, 4), "int8"), 0, 0, 1.0, 1.0,
                      kernel_size=(3, 3), channels=4, data_layout="NCWH")


def test_simulated_ops_lowering_and_text():
    """qnn.simulated_quantize / _dequantize: the constructor's reshape(-1) of constant parameters
    folds (FoldConstant) -- no op, no MRT name -- and the constants ride with the node; graph-tensor
    parameters stay tensors the node reads; Relay text round-trips to the same plan."""
    from tachikoma_amd.relay.build_module import lower
    x = relay.var("x", shape=(2, 3, 4), dtype="float32")
    y = qnn.op.simulated_quantize(x, relay.const(np.array([0.5, 0.25, 0.125], np.float32)), relay.const(3), axis=1,
                                  out_dtype="int8")
    code = relay.var("code", shape=(1,), dtype="int32")
    zp = relay.var("zp", shape=(2,), dtype="int32")
    z = qnn.op.simulated_dequantize(y, relay.const(0.5), zp, axis=-1, in_dtype=code)
    mod = relay.IRModule.from_expr(relay.Function([x, code, zp], z))
    plan = lower(mod, {})
    assert [o.op for o in plan.ops] == ["qnn.simulated_quantize", "reshape", "qnn.simulated_dequantize"]
    q, r, d = plan.ops
    assert q.name == "%0" and q.attrs["axis"] == 1 and q.attrs["sources"] == {"dtype_code": -1, "scales": -1,
                                                                                  "zero_points": -1}
    np.testing.assert_array_equal(q.consts["dtype_code"], [1])
    np.testing.assert_array_equal(q.consts["scales"], np.array([0.5, 0.25, 0.125], np.float32))
    assert r.inputs == ["zp"] and d.inputs == ["%0", "code", "%1"]
    assert d.attrs["axis"] == 2 and d.attrs["sources"] == {"dtype_code": 1, "scales": -1, "zero_points": 2}
    assert d.attrs["n_zero_points"] == 2 and "zero_points" not in d.consts
    again = lower(relay.parse(mod.astext()), {})
    assert [o.describe() for o in again.ops] == [o.describe() for o in plan.ops]
    # the oracle walker folds the same reshape and names the same records
    rng = np.random.default_rng(2)
    inputs = {"x": rng.standard_normal((2, 3, 4)).astype(np.float32) * 9, "code": np.array([2], np.int32),
              "zp": np.array([1, -1], np.int32)}
    rec = graph_ref.calibrate(mod, {}, inputs)
    assert sorted(rec) == sorted(["x", "code", "zp", "%0", "%1", "%2"])
    e0 = ref.simulated_quantize(inputs["x"], 1, [0.5, 0.25, 0.125], [3], axis=1)
    np.testing.assert_array_equal(rec["%0"], e0)
    np.testing.assert_array_equal(rec["%2"], ref.simulated_dequantize(e0, 2, [0.5], [1, -1], axis=-1))
    with pytest.raises(TypeError):
        qnn.op.simulated_quantize(relay.var("i", shape=(2,), dtype="int8"), 0.5, 0)
    with pytest.raises(ValueError):
        qnn.op.simulated_quantize(x, 0.5, 0, out_dtype="int16")


def test_simulated_ops_build_keeps_parameter_constants():
    """relay.build lifts tensor constants of ordinary ops into params; the simulated ops' reshaped
    per-channel parameters must stay constants (folded, no reshape op, no record)."""
    x = relay.var("x", shape=(2, 7, 3), dtype="float32")
    s = np.linspace(0.1, 0.7, 7).astype(np.float32)
    q = qnn.op.simulated_quantize(x, relay.const(s), relay.const(np.arange(7, dtype=np.int32)), axis=1)
    lib = build(relay.IRModule.from_expr(q), target="mi355x", params={})
    assert [o.op for o in lib.plan.ops] == ["qnn.simulated_quantize"]
    np.testing.assert_array_equal(lib.plan.ops[0].consts["scales"], s)

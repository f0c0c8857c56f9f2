"""The pre-quantized QNN ops on the MI355X, bit-exact vs the CPU oracle.

qnn.quantize / qnn.dequantize / qnn.concatenate / qnn.mul / qnn.subtract (and broadcast / per-axis
qnn.add), NHWC data with HWIO / OHWI / HWOI kernels (incl. the depthwise-multiplier form) for
qnn.conv2d, and a frontend-shaped QNN graph written as Relay text (quantize -> NHWC conv block ->
concatenate -> dequantize).  Every op runs as its HIP kernel through the module's C-ABI node loop
and every trace record is compared with oracle/graph_ref.py; the reference's literal KATs
(tests/golden/qnn_kats.json) are checked against the device output directly.
"""
import numpy as np
import pytest

from oracle import graph_ref
from oracle import qnn_ref as ref
from tachikoma_amd import relay
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.relay import qnn
from tachikoma_amd.trace_format import read_trace
from tests.golden_util import load_array, load_cases

pytestmark = pytest.mark.gpu


def _trace(expr, inputs, tmp_path, params=None):
    """Build, run once with capture and return (trace records, oracle records)."""
    mod = relay.IRModule.from_expr(expr)
    lib = relay.build(mod, target="mi355x", params=params or {})
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input(**inputs)
    path = str(tmp_path / "t.tkt")
    m.dump_trace(path)
    tr = read_trace(path, copy=True)
    exp = graph_ref.calibrate(mod, params or {}, inputs)
    return tr.records, exp


def _check(records, expected):
    assert set(records) == set(expected)
    for name, e in expected.items():
        g = records[name]
        assert g.shape == e.shape and g.dtype == e.dtype, (name, g.shape, e.shape, g.dtype, e.dtype)
        if not np.array_equal(g.view(np.uint8) if g.dtype == np.float32 else g,
                              e.view(np.uint8) if e.dtype == np.float32 else e):
            bad = np.argwhere(g != e)
            raise AssertionError(f"record {name}: {len(bad)} mismatches, first at {tuple(bad[0])}: "
                                 f"{g[tuple(bad[0])]} vs {e[tuple(bad[0])]}")


def _c(v, dtype):
    return relay.const(np.array(v, dtype=dtype)) if isinstance(v, list) else relay.const(v, dtype)


# ---------------------------------------------------------------- the reference's KATs

@pytest.mark.parametrize("case", load_cases("qnn.quantize"), ids=lambda c: c["name"])
def test_quantize_kat(device, tmp_path, case):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    if x.ndim == 0:
        pytest.skip("rank-0 graph inputs are not traced tensors here (covered by the oracle KAT)")
    v = relay.var("x", x.shape, "float32")
    e = qnn.op.quantize(v, _c(a["output_scale"], "float32"), _c(a["output_zero_point"], "int32"), axis=a["axis"],
                        out_dtype=a["out_dtype"])
    rec, exp = _trace(e, {"x": x}, tmp_path)
    _check(rec, exp)
    np.testing.assert_array_equal(rec["%0"], load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.dequantize"), ids=lambda c: c["name"])
def test_dequantize_kat(device, tmp_path, case):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    if x.ndim == 0:
        pytest.skip("rank-0 graph inputs are not traced tensors here (covered by the oracle KAT)")
    v = relay.var("x", x.shape, str(x.dtype))
    e = qnn.op.dequantize(v, _c(a["input_scale"], "float32"), _c(a["input_zero_point"], "int32"), axis=a["axis"])
    rec, exp = _trace(e, {"x": x}, tmp_path)
    _check(rec, exp)
    np.testing.assert_array_equal(rec["%0"], load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.concatenate"), ids=lambda c: c["name"])
def test_concatenate_kat(device, tmp_path, case):
    a = case["attrs"]
    xs = [load_array(d) for d in case["inputs"]["data"]]
    vs = [relay.var(f"x{i}", x.shape, str(x.dtype)) for i, x in enumerate(xs)]
    e = qnn.op.concatenate(vs, [np.float32(s) for s in a["input_scales"]],
                           [np.int32(z) for z in a["input_zero_points"]], np.float32(a["output_scale"]),
                           np.int32(a["output_zero_point"]), axis=a["axis"])
    rec, exp = _trace(e, {f"x{i}": x for i, x in enumerate(xs)}, tmp_path)
    _check(rec, exp)
    np.testing.assert_array_equal(rec["%0"], load_array(case["expected"]))


@pytest.mark.parametrize("op", ["qnn.mul", "qnn.subtract", "qnn.add"])
def test_binary_kats(device, tmp_path, op):
    fn = {"qnn.mul": qnn.op.mul, "qnn.subtract": qnn.op.subtract, "qnn.add": qnn.op.add}[op]
    for case in load_cases(op):
        a = case["attrs"]
        x, y = load_array(case["inputs"]["lhs"]), load_array(case["inputs"]["rhs"])
        vx, vy = relay.var("x", x.shape, str(x.dtype)), relay.var("y", y.shape, str(y.dtype))
        # a multiply-then-subtract pair keeps the binary ops off the fused residual-join kernels
        e = fn(vx, vy, np.float32(a["lhs_scale"]), np.int32(a["lhs_zero_point"]), np.float32(a["rhs_scale"]),
               np.int32(a["rhs_zero_point"]), np.float32(a["output_scale"]), np.int32(a["output_zero_point"]))
        rec, exp = _trace(e, {"x": x, "y": y}, tmp_path)
        _check(rec, exp)
        np.testing.assert_array_equal(rec["%0"], load_array(case["expected"]), err_msg=case["name"])


# ---------------------------------------------------------------- random sweeps

@pytest.mark.parametrize("out_dtype", ["int8", "uint8", "int16", "int32"])
@pytest.mark.parametrize("per_axis", [False, True])
def test_quantize_dequantize_random(device, tmp_path, out_dtype, per_axis):
    rng = np.random.default_rng(11)
    shape = (3, 7, 5, 9)
    lo, hi = np.iinfo(out_dtype).min, np.iinfo(out_dtype).max
    s = rng.uniform(0.001, 0.2, 7).astype(np.float32) if per_axis else np.float32(0.037)
    z = rng.integers(-20, 20, 7).astype(np.int32) if per_axis else np.int32(-3)
    if out_dtype == "uint8":
        z = np.abs(z) + 100
    span = float(hi - lo) * (0.3 if out_dtype != "int32" else 1e-6)
    x = (rng.standard_normal(shape) * span * 0.04).astype(np.float32)
    # exact halves (round-half-away), values past both clip bounds and -0.0
    x.reshape(-1)[:6] = [0.5 * 0.037, -0.5 * 0.037, 1e9, -1e9, -0.0, 2.5 * 0.037]
    v = relay.var("x", shape, "float32")
    q = qnn.op.quantize(v, relay.const(s), relay.const(z), axis=1, out_dtype=out_dtype)
    d = qnn.op.dequantize(q, relay.const(s), relay.const(z), axis=1)
    rec, exp = _trace(d, {"x": x}, tmp_path)
    _check(rec, exp)


@pytest.mark.parametrize("dtype", ["int8", "uint8", "int16", "int32"])
def test_concatenate_random(device, tmp_path, dtype):
    rng = np.random.default_rng(5)
    info = np.iinfo(dtype)
    shapes = [(2, 3, 4, 5), (2, 1, 4, 5), (2, 6, 4, 5), (2, 2, 4, 5), (2, 5, 4, 5)]
    xs = [rng.integers(max(info.min, -2 ** 20), min(info.max, 2 ** 20) + 1, sh).astype(dtype) for sh in shapes]
    scales = [np.float32(0.05), np.float32(0.1), np.float32(0.05), np.float32(0.0123), np.float32(0.5)]
    zps = [np.int32(0), np.int32(3), np.int32(-2), np.int32(0), np.int32(7)]
    vs = [relay.var(f"x{i}", sh, dtype) for i, sh in enumerate(shapes)]
    e = qnn.op.concatenate(vs, scales, zps, np.float32(0.05), np.int32(0), axis=1)
    rec, exp = _trace(e, {f"x{i}": x for i, x in enumerate(xs)}, tmp_path)
    _check(rec, exp)
    # axis = -1 (a trailing-axis concatenation)
    e = qnn.op.concatenate(vs[:1] + [relay.var("y", (2, 3, 4, 2), dtype)], scales[:2], zps[:2], np.float32(0.1),
                           np.int32(1), axis=-1)
    y = rng.integers(max(info.min, -2 ** 20), min(info.max, 2 ** 20) + 1, (2, 3, 4, 2)).astype(dtype)
    rec, exp = _trace(e, {"x0": xs[0], "y": y}, tmp_path)
    _check(rec, exp)


@pytest.mark.parametrize("op", ["qnn.add", "qnn.subtract", "qnn.mul"])
@pytest.mark.parametrize("dtype", ["int8", "uint8", "int32"])
def test_binary_broadcast_random(device, tmp_path, op, dtype):
    rng = np.random.default_rng(17)
    fn = {"qnn.add": qnn.op.add, "qnn.subtract": qnn.op.subtract, "qnn.mul": qnn.op.mul}[op]
    info = np.iinfo(dtype)
    lim = 2 ** 12 if dtype == "int32" else None
    ri = lambda sh: rng.integers(info.min if lim is None else -lim, (info.max if lim is None else lim) + 1,  # noqa
                                 sh).astype(dtype)
    zp0 = 128 if dtype == "uint8" else 0
    for lshape, rshape in (((2, 3, 4, 5), (2, 3, 4, 5)), ((2, 3, 4, 5), (3, 1, 1)), ((1, 3, 1, 5), (2, 1, 4, 1)),
                           ((4, 5), (5,))):
        x, y = ri(lshape), ri(rshape)
        vx, vy = relay.var("x", lshape, dtype), relay.var("y", rshape, dtype)
        e = fn(vx, vy, np.float32(0.021), np.int32(zp0 + 3), np.float32(0.017), np.int32(zp0 - 5),
               np.float32(0.05 if op != "qnn.mul" else 0.3), np.int32(zp0 + 1))
        rec, exp = _trace(e, {"x": x, "y": y}, tmp_path)
        _check(rec, exp)


@pytest.mark.parametrize("op", ["qnn.add", "qnn.subtract", "qnn.mul"])
def test_binary_per_axis_random(device, tmp_path, op):
    """Per-axis scales / zero points (RequantizeOrUpcast along each operand's axis; qnn.mul's
    per-channel branch with equal axes)."""
    rng = np.random.default_rng(23)
    fn = {"qnn.add": qnn.op.add, "qnn.subtract": qnn.op.subtract, "qnn.mul": qnn.op.mul}[op]
    shape = (2, 6, 4, 5)
    x = rng.integers(-128, 128, shape).astype(np.int8)
    y = rng.integers(-128, 128, shape).astype(np.int8)
    ls = rng.uniform(0.005, 0.05, 6).astype(np.float32)
    rs = rng.uniform(0.005, 0.05, 6).astype(np.float32)
    lz = rng.integers(-4, 5, 6).astype(np.int32)
    rz = rng.integers(-4, 5, 6).astype(np.int32)
    vx, vy = relay.var("x", shape, "int8"), relay.var("y", shape, "int8")
    e = fn(vx, vy, relay.const(ls), relay.const(lz), relay.const(rs), relay.const(rz), np.float32(0.04 if op != "qnn.mul" else 0.002),
           np.int32(2), lhs_axis=1, rhs_axis=1)
    rec, exp = _trace(e, {"x": x, "y": y}, tmp_path)
    _check(rec, exp)


def test_binary_tonearest_config(device, tmp_path):
    """The requantize inside qnn.mul / qnn.subtract follows the requantize_config in effect when the
    op is built (Requantize with rounding "None", qnn/utils.h:106-122)."""
    rng = np.random.default_rng(29)
    x = rng.integers(-128, 128, (3, 64)).astype(np.int8)
    y = rng.integers(-128, 128, (3, 64)).astype(np.int8)
    vx, vy = relay.var("x", x.shape, "int8"), relay.var("y", y.shape, "int8")
    with qnn.op.requantize_config(rounding="TONEAREST"):
        m = qnn.op.mul(vx, vy, np.float32(0.02), np.int32(1), np.float32(0.03), np.int32(-1), np.float32(0.25),
                       np.int32(0))
        s = qnn.op.subtract(m, vy, np.float32(0.25), np.int32(0), np.float32(0.03), np.int32(-1), np.float32(0.07),
                            np.int32(3))
    rec, exp = _trace(s, {"x": x, "y": y}, tmp_path)
    _check(rec, exp)


# ---------------------------------------------------------------- conv layouts

def _conv_case(rng, data_layout, kernel_layout, c, o, k, groups, mult=1, dtype="int8", zw_vec=False, stride=1, pad=1):
    n, h, w = 2, 9, 7
    lo, hi = (0, 256) if dtype == "uint8" else (-128, 128)
    if mult > 1:
        wo = (c, mult, k, k)  # the depthwise-multiplier form (C, M, KH, KW)
    else:
        wo = (o, c // groups, k, k)
    wt = rng.integers(lo, hi, wo).astype(dtype)
    wt_l = np.ascontiguousarray(wt.transpose(["OIHW".index(ch) for ch in kernel_layout]))
    x = rng.integers(lo, hi, (n, c, h, w)).astype(dtype)
    x_l = x if data_layout == "NCHW" else np.ascontiguousarray(x.transpose(0, 2, 3, 1))
    zw = relay.const(rng.integers(-3, 4, wo[0]).astype(np.int32)) if zw_vec else relay.const(2, "int32")
    vx = relay.var("x", x_l.shape, dtype)
    vw = relay.var("w", wt_l.shape, dtype)
    za = 131 if dtype == "uint8" else -3
    e = qnn.op.conv2d(vx, vw, relay.const(za, "int32"), zw, relay.const(0.1), relay.const(0.1), kernel_size=(k, k),
                      channels=c * mult if mult > 1 else o, strides=(stride, stride), padding=(pad, pad),
                      groups=groups, data_layout=data_layout, kernel_layout=kernel_layout)
    return e, {"x": x_l}, {"w": wt_l}, (x, wt)


@pytest.mark.parametrize("data_layout,kernel_layout", [("NHWC", "HWIO"), ("NHWC", "OHWI"), ("NHWC", "HWOI"),
                                                       ("NCHW", "HWIO"), ("NHWC", "OIHW")])
@pytest.mark.parametrize("c,o,k,groups", [(16, 32, 3, 1), (3, 8, 5, 1), (64, 64, 1, 1), (8, 8, 3, 8), (12, 24, 3, 3)])
def test_conv_layouts(device, tmp_path, data_layout, kernel_layout, c, o, k, groups):
    rng = np.random.default_rng(c * 31 + o + k)
    e, inputs, params, (x, wt) = _conv_case(rng, data_layout, kernel_layout, c, o, k, groups, zw_vec=(groups == 1))
    rec, exp = _trace(e, inputs, tmp_path, params)
    _check(rec, exp)
    # the NCHW / OIHW contraction of the same operands, in the data layout (the reference's own
    # layout test compares against nn.conv2d of the shifted operands in each layout)
    zw = e.args[3].data
    nchw = ref.qnn_conv2d(x, wt, e.args[2].data, zw, padding=(1, 1, 1, 1),
                          groups=groups) if k != 5 else None
    if nchw is not None:
        got = rec["%0"] if data_layout == "NCHW" else rec["%0"].transpose(0, 3, 1, 2)
        np.testing.assert_array_equal(got, nchw)


@pytest.mark.parametrize("data_layout,kernel_layout", [("NCHW", "OIHW"), ("NHWC", "HWOI")])
@pytest.mark.parametrize("dtype", ["int8", "uint8"])
def test_conv_depthwise_multiplier(device, tmp_path, data_layout, kernel_layout, dtype):
    """Conv2DRel's depthwise weight (C, M, KH, KW): output channel c * M + m (test_op_qnn_conv2d.py:
    954-1066), per-channel kernel zero points along C."""
    rng = np.random.default_rng(41)
    e, inputs, params, _ = _conv_case(rng, data_layout, kernel_layout, 4, 8, 3, 4, mult=2, dtype=dtype, zw_vec=True,
                                      pad=0)
    rec, exp = _trace(e, inputs, tmp_path, params)
    _check(rec, exp)


QNN_TEXT = """#[version = "0.0.5"]
def @main(%x: Tensor[(2, 14, 14, 16), float32], %w: Tensor[(3, 3, 16, 32), int8], %b: Tensor[(32), int32],
          %y: Tensor[(2, 14, 14, 8), int8]) {
  %0 = qnn.quantize(%x, 0.05f, -3, out_dtype="int8");
  %1 = qnn.conv2d(%0, %w, -3, 0, 0.05f, 0.02f, padding=[1, 1, 1, 1], channels=32, kernel_size=[3, 3],
                  data_layout="NHWC", kernel_layout="HWIO", out_dtype="int32");
  %2 = nn.bias_add(%1, %b, axis=3);
  %3 = qnn.requantize(%2, 0.001f, 0, 0.1f, 2, axis=3, out_dtype="int8");
  %4 = clip(%3, a_min=-128f, a_max=127f);
  %5 = (%4, %y);
  %6 = qnn.concatenate(%5, (0.1f, 0.07f), (2, -1), 0.09f, 1, axis=3);
  %7 = qnn.mul(%6, %6, 0.09f, 1, 0.09f, 1, 0.2f, -4);
  %8 = qnn.subtract(%7, %6, 0.2f, -4, 0.09f, 1, 0.15f, 0);
  qnn.dequantize(%8, 0.15f, 0)
}
"""


def test_frontend_qnn_graph_text(device, tmp_path):
    """A QNN graph the way a frontend emits it, as Relay text: float32 input quantize -> NHWC / HWIO
    conv -> bias / requantize / clip on axis 3 -> concatenate with a second branch -> mul -> subtract
    -> float32 dequantize.  Parsed, built and traced; every record bit-exact vs the oracle."""
    mod = relay.parse(QNN_TEXT)
    rng = np.random.default_rng(3)
    params = {"w": rng.integers(-128, 128, (3, 3, 16, 32)).astype(np.int8),
              "b": rng.integers(-5000, 5000, 32).astype(np.int32)}
    inputs = {"x": rng.standard_normal((2, 14, 14, 16)).astype(np.float32) * 3,
              "y": rng.integers(-128, 128, (2, 14, 14, 8)).astype(np.int8)}
    lib = relay.build(mod, target="mi355x", params=params)
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input(**inputs)
    path = str(tmp_path / "qnn.tkt")
    m.dump_trace(path)
    tr = read_trace(path, copy=True)
    exp = graph_ref.calibrate(mod, params, inputs)
    _check(tr.records, exp)
    assert [o["op"] for o in tr.meta["ops"]] == ["qnn.quantize", "qnn.conv2d", "nn.bias_add", "qnn.requantize",
                                                 "clip", "qnn.concatenate", "qnn.mul", "qnn.subtract",
                                                 "qnn.dequantize"]
    # the replayed-graph run gives the same image
    m.module.use_graph = True
    m.run(trace=True)
    m.trace_capture().synchronize()
    tr2 = read_trace(m.trace_capture().bytes(), copy=True)
    _check(tr2.records, exp)


# ---------------------------------------------------------------- round 5: leaky_relu, the unary
# table lookups, batch_matmul, conv2d_transpose

@pytest.mark.parametrize("case", load_cases("qnn.leaky_relu"), ids=lambda c: c["name"])
def test_leaky_relu_kat(device, tmp_path, case):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    v = relay.var("x", x.shape, str(x.dtype))
    e = qnn.op.leaky_relu(v, a["alpha"], np.float32(a["input_scale"]), np.int32(a["input_zero_point"]),
                          np.float32(a["output_scale"]), np.int32(a["output_zero_point"]))
    rec, exp = _trace(e, {"x": x}, tmp_path)
    _check(rec, exp)
    np.testing.assert_array_equal(rec["%0"], load_array(case["expected"]))


@pytest.mark.parametrize("dtype", ["int8", "uint8"])
@pytest.mark.parametrize("alpha,s_in,z_in,s_out,z_out,rounding", [
    (0.1, 0.05, 3, 0.05, 3, "UPWARD"),        # same params: RequantizeOrUpcast casts
    (0.25, 0.05, -7, 0.11, 9, "UPWARD"),
    (0.5, 0.125, 60, 0.6, 17, "TONEAREST"),   # alpha 0.5: the power-of-two fixed_point_multiply
    (0.333, 0.02, 0, 0.0625, -4, "TONEAREST"),
    (0.9, 0.125, 60, 0.25, 0, "UPWARD"),      # 1 - alpha = 0.1
])
def test_leaky_relu_random(device, tmp_path, dtype, alpha, s_in, z_in, s_out, z_out, rounding):
    rng = np.random.default_rng(int(alpha * 1000) + 7)
    lo, hi = (0, 256) if dtype == "uint8" else (-128, 128)
    x = rng.integers(lo, hi, (3, 5, 67)).astype(dtype)
    v = relay.var("x", x.shape, dtype)
    with qnn.op.requantize_config(rounding=rounding):
        e = qnn.op.leaky_relu(v, alpha, np.float32(s_in), np.int32(z_in), np.float32(s_out), np.int32(z_out))
    rec, exp = _trace(e, {"x": x}, tmp_path)
    _check(rec, exp)


@pytest.mark.parametrize("case", load_cases("qnn.unary"), ids=lambda c: c["name"])
def test_unary_kat(device, tmp_path, case):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    v = relay.var("x", x.shape, str(x.dtype))
    e = getattr(qnn.op, a["unary_op"].split(".")[1])(v, np.float32(a["scale"]), np.int32(a["zero_point"]),
                                                     np.float32(a["output_scale"]), np.int32(a["output_zero_point"]))
    rec, exp = _trace(e, {"x": x}, tmp_path)
    _check(rec, exp)
    np.testing.assert_array_equal(rec["%0"], load_array(case["expected"]))


@pytest.mark.parametrize("op", list(qnn.op.UNARY_OPS))
@pytest.mark.parametrize("dtype", ["int8", "uint8"])
def test_unary_every_pattern_and_ragged(device, tmp_path, op, dtype):
    """Every 8-bit pattern (the whole table) in a ragged tensor (the 16-byte path and its tail), with
    asymmetric params, bit-exact vs the oracle's table (same numpy functions)."""
    rng = np.random.default_rng(hash(op) % 1000)
    base = np.arange(256, dtype=np.uint8).view(dtype)
    x = np.concatenate([base, rng.integers(0, 256, 1000 - 256).astype(np.uint8).view(dtype)]).reshape(8, 125)
    v = relay.var("x", x.shape, dtype)
    e = getattr(qnn.op, op.split(".")[1])(v, np.float32(0.037), np.int32(5 if dtype == "uint8" else -3),
                                          np.float32(0.021), np.int32(100 if dtype == "uint8" else 2))
    rec, exp = _trace(e, {"x": x}, tmp_path)
    _check(rec, exp)


@pytest.mark.parametrize("case", load_cases("qnn.batch_matmul"), ids=lambda c: c["name"])
def test_batch_matmul_kat(device, tmp_path, case):
    a = case["attrs"]
    x, y = load_array(case["inputs"]["x"]), load_array(case["inputs"]["y"])
    vx, vy = relay.var("x", x.shape, "int8"), relay.var("y", y.shape, "int8")
    e = qnn.op.batch_matmul(vx, vy, np.int32(a["x_zero_point"]), np.int32(a["y_zero_point"]), np.float32(a["x_scale"]),
                            np.float32(a["y_scale"]))
    if "requantize" in case:
        r = case["requantize"]
        e = qnn.op.requantize(e, np.float32(r["input_scale"]), np.int32(0), np.float32(r["output_scale"]),
                              np.int32(r["output_zero_point"]), out_dtype=r["out_dtype"])
    rec, exp = _trace(e, {"x": x, "y": y}, tmp_path)
    _check(rec, exp)
    np.testing.assert_array_equal(rec[sorted(rec, key=lambda k: int(k[1:]) if k[1:].isdigit() else -1)[-1]],
                                  load_array(case["expected"]))


@pytest.mark.parametrize("bx,by,m,n,k,dtype,zx,zy", [
    (4, 4, 33, 70, 96, "int8", 3, -5),
    (1, 6, 128, 64, 64, "uint8", 128, 120),   # x broadcast over y's batch
    (5, 1, 17, 9, 200, "int8", 0, 7),          # y broadcast
    (12, 12, 128, 128, 64, "int8", -1, 0),     # attention-shaped
])
def test_batch_matmul_random(device, tmp_path, bx, by, m, n, k, dtype, zx, zy):
    rng = np.random.default_rng(bx * 100 + m)
    lo, hi = (0, 256) if dtype == "uint8" else (-128, 128)
    x = rng.integers(lo, hi, (bx, m, k)).astype(dtype)
    y = rng.integers(lo, hi, (by, n, k)).astype(dtype)
    vx, vy = relay.var("x", x.shape, dtype), relay.var("y", y.shape, dtype)
    e = qnn.op.batch_matmul(vx, vy, np.int32(zx), np.int32(zy), np.float32(0.1), np.float32(0.2))
    rec, exp = _trace(e, {"x": x, "y": y}, tmp_path)
    _check(rec, exp)


@pytest.mark.parametrize("ds,ws,zd,zw,st,pad,opad,groups,dtype,dl,kl", [
    # test_op_qnn_conv2_transpose.py's cases
    ((2, 1, 2, 4), (1, 3, 2, 2), 0, 0, (1, 1), (0, 0), (0, 0), 1, "uint8", "NCHW", "IOHW"),
    ((2, 4, 2, 4), (4, 3, 2, 2), 0, 1, (1, 1), (0, 0), (0, 0), 1, "int8", "NCHW", "IOHW"),
    ((2, 4, 2, 4), (4, 3, 2, 2), 5, 3, (1, 1), (0, 0), (0, 0), 1, "uint8", "NCHW", "IOHW"),
    ((1, 4, 2, 2), (4, 3, 2, 2), 8, 5, (1, 1), (1, 1), (0, 0), 1, "uint8", "NCHW", "IOHW"),
    ((2, 2, 4, 4), (2, 2, 3, 4), 5, 3, (1, 1), (0, 0), (0, 0), 1, "uint8", "NHWC", "HWOI"),
    ((2, 8, 6, 4), (2, 2, 3, 4), 8, 3, (1, 1), (1, 1, 2, 2), (0, 0), 1, "uint8", "NHWC", "HWOI"),
    # strides, output padding, groups, a per-channel kernel zero point
    ((2, 16, 7, 7), (16, 8, 3, 3), 2, -1, (2, 2), (1, 1), (1, 1), 1, "int8", "NCHW", "IOHW"),
    ((1, 12, 5, 6), (12, 4, 4, 4), -3, 2, (2, 3), (1, 0, 2, 1), (1, 2), 3, "int8", "NCHW", "IOHW"),
    ((2, 4, 3, 3), (4, 3, 2, 2), 1, [1, -2, 3], (2, 2), (0, 0), (0, 0), 1, "uint8", "NCHW", "IOHW"),
    ((1, 6, 6, 8), (3, 3, 8, 5), 4, 1, (2, 2), (1, 1), (0, 0), 1, "int8", "NHWC", "HWIO"),
])
def test_conv2d_transpose(device, tmp_path, ds, ws, zd, zw, st, pad, opad, groups, dtype, dl, kl):
    rng = np.random.default_rng(sum(ds) + sum(ws))
    lo, hi = (0, 256) if dtype == "uint8" else (-128, 128)
    x = rng.integers(lo, hi, ds).astype(dtype)
    w = rng.integers(lo, hi, ws).astype(dtype)
    vx, vw = relay.var("x", ds, dtype), relay.var("w", ws, dtype)
    e = qnn.op.conv2d_transpose(vx, vw, np.int32(zd), _c(zw, "int32"), np.float32(0.5), np.float32(0.25), strides=st,
                                padding=pad, groups=groups, data_layout=dl, kernel_layout=kl, output_padding=opad)
    rec, exp = _trace(e, {"x": x}, tmp_path, params={"w": w})
    _check(rec, exp)


def test_round5_ops_in_one_graph_text(device, tmp_path):
    """A generator-shaped QNN graph -- conv2d_transpose -> requantize -> leaky_relu -> hardswish ->
    batch_matmul over the flattened maps -- built from constructors, printed as Relay text, parsed back
    and traced (plain and as a replayed HIP graph), every record bit-exact vs the oracle."""
    rng = np.random.default_rng(5)
    x = rng.integers(-128, 128, (2, 8, 4, 4)).astype(np.int8)
    w = rng.integers(-128, 128, (8, 4, 3, 3)).astype(np.int8)
    vx, vw = relay.var("x", x.shape, "int8"), relay.var("w", w.shape, "int8")
    ct = qnn.op.conv2d_transpose(vx, vw, np.int32(1), np.int32(0), np.float32(0.05), np.float32(0.01), strides=(2, 2),
                                 padding=(1, 1), output_padding=(1, 1))
    rq = qnn.op.requantize(ct, np.float32(0.0005), np.int32(0), np.float32(0.1), np.int32(-2), out_dtype="int8")
    lr = qnn.op.leaky_relu(rq, 0.2, np.float32(0.1), np.int32(-2), np.float32(0.08), np.int32(0))
    hs = qnn.op.hardswish(lr, np.float32(0.08), np.int32(0), np.float32(0.05), np.int32(-10))
    r3 = relay.reshape(hs, (2, 4, 64))
    bm = qnn.op.batch_matmul(r3, r3, np.int32(-10), np.int32(-10), np.float32(0.05), np.float32(0.05))
    mod = relay.IRModule.from_expr(bm)
    text = mod.astext()
    assert "qnn.conv2d_transpose" in text and "qnn.leaky_relu" in text and "qnn.hardswish" in text
    mod2 = relay.parse(text)
    exp = graph_ref.calibrate(mod2, {"w": w}, {"x": x})
    for use_graph in (False, True):
        lib = relay.build(mod2, target="mi355x", params={"w": w})
        m = graph_executor.GraphModule(lib["default"]())
        m.module.use_graph = use_graph
        m.set_input(x=x)
        path = str(tmp_path / f"g{int(use_graph)}.tkt")
        m.dump_trace(path)
        _check(read_trace(path, copy=True).records, exp)
        m.close()


# ---------------------------------------------------------------- simulated (de)quantize

@pytest.mark.parametrize("dt", ["int8", "uint8", "int32", "disable"])
@pytest.mark.parametrize("axis,ns,nz", [(1, 7, 7), (-1, 1, 1), (2, 2, 3)])
def test_simulated_ops_random(device, tmp_path, dt, axis, ns, nz):
    """qnn.simulated_quantize -> qnn.simulated_dequantize with constant parameters: per-tensor,
    per-channel, and fewer values than the axis has (taken modulo their count)."""
    rng = np.random.default_rng(13)
    shape = (3, 7, 5, 9)
    s = rng.uniform(0.01, 0.3, ns).astype(np.float32)
    z = rng.integers(-10, 10, nz).astype(np.int32) + (100 if dt == "uint8" else 0)
    x = (rng.standard_normal(shape) * 40).astype(np.float32)
    # exact halves, values past every clip bound, -0.0 (all in channel 0 of the three axes)
    x.reshape(-1)[:6] = [0.5 * s[0], -0.5 * s[0], 1e10, -1e10, -0.0, 2.5 * s[0]]
    v = relay.var("x", shape, "float32")
    q = qnn.op.simulated_quantize(v, relay.const(s), relay.const(z), axis=axis, out_dtype=dt)
    d = qnn.op.simulated_dequantize(q, relay.const(s), relay.const(z), axis=axis, in_dtype=dt)
    rec, exp = _trace(d, {"x": x}, tmp_path)
    _check(rec, exp)


def test_simulated_ops_dynamic_params(device, tmp_path):
    """The dtype code, scales and zero points as graph inputs (test_op_qnn_simulated_quantize.py's
    dynamic dtype / dynamic channels cases): one module, run with several codes and parameter sets
    without rebuilding; each trace bit-exact vs the oracle."""
    rng = np.random.default_rng(17)
    shape = (2, 5, 8)
    x = (rng.standard_normal(shape) * 30).astype(np.float32)
    vx = relay.var("x", shape, "float32")
    vs, vz, vc = relay.var("scale", (2,), "float32"), relay.var("zp", (2,), "int32"), relay.var("dtype", (1,), "int32")
    q = qnn.op.simulated_quantize(vx, vs, vz, axis=1, out_dtype=vc)
    d = qnn.op.simulated_dequantize(q, vs, vz, axis=1, in_dtype=vc)
    mod = relay.IRModule.from_expr(d)
    m = graph_executor.GraphModule(relay.build(mod, target="mi355x", params={})["default"]())
    for code, s, z in [(2, [0.5, 0.25], [127, 123]), (3, [0.5, 0.5], [127, 127]), (1, [0.1, 0.3], [-3, 4]),
                       (0, [0.5, 0.25], [1, 2])]:
        inputs = {"x": x, "scale": np.array(s, np.float32), "zp": np.array(z, np.int32),
                  "dtype": np.array([code], np.int32)}
        m.set_input(**inputs)
        path = str(tmp_path / f"t{code}.tkt")
        m.dump_trace(path)
        _check(read_trace(path, copy=True).records, graph_ref.calibrate(mod, {}, inputs))

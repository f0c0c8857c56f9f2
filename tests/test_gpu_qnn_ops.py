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

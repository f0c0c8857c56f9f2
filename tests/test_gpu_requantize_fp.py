"""qnn.requantize with compute_dtype float32 / float64 on the MI355X (RequantizeLowerFP<Bits>,
src/relay/qnn/op/requantize.cc:293-373, with the non-SSE4.1 Upward / Tonearest forms of :127-173),
bit-exact vs the CPU oracle (oracle/qnn_ref.py requantize_fp).

* the reference's literal requantize KATs (tests/golden/qnn_kats.json), which its own test runs
  under all three compute dtypes against the same goldens (test_op_qnn_requantize.py:25), through
  the C-ABI entry tk_requantize_fp;
* seeded random int32 data over the whole int32 range, per-tensor and per-axis, both roundings,
  both widths, several in / out dtypes -- including multipliers > 1 whose products leave the int32
  range (x86 fptosi's INT_MIN, then the clip) and values where float32 loses integer precision
  (where the float forms and the int64 form really differ);
* graphs built under requantize_config(compute_dtype=...): LeNet-5 (conv / dense blocks run
  unfused, the requantize on tk_requantize_fp) and a qnn.add / subtract / mul graph with per-axis
  scales on tk_qnn_binary_fp, every trace record compared with oracle/graph_ref.py.
"""
import ctypes

import numpy as np
import pytest

from oracle import graph_ref
from oracle import qnn_ref as ref
from tachikoma_amd import _lib, relay, zoo
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.relay import qnn
from tachikoma_amd.relay.build_module import fp_requantize_plan
from tachikoma_amd.trace_format import read_trace
from tests import tk_gpu
from tests.golden_util import load_array, load_cases, scale_const

pytestmark = pytest.mark.gpu


def requantize_fp_gpu(x, s_in, zp_in, s_out, zp_out, axis, rounding, out_dtype, bits):
    """One tk_requantize_fp launch on numpy data (zero points: int or per-axis vector)."""
    lib = _lib.load()
    xd = tk_gpu.dev(x)
    out = tk_gpu.empty(x.shape, out_dtype)
    a = _lib.tk_requantize_fp_attrs()
    a.bits = bits
    a.rounding = _lib.TK_ROUND_UPWARD if rounding == "UPWARD" else _lib.TK_ROUND_TONEAREST
    nd = x.ndim
    a.axis = axis if axis >= 0 else (nd + axis if nd else 0)
    scaled, m, ms = fp_requantize_plan(s_in, s_out)
    a.scaled, a.multiplier = scaled, m
    keep = []
    if ms is not None:
        keep.append(tk_gpu.dev(ms))
        a.multipliers = keep[-1].data_ptr()
    zp = np.asarray(zp_in, np.int32)
    if zp.ndim:
        keep.append(tk_gpu.dev(zp.reshape(-1)))
        a.input_zero_points = keep[-1].data_ptr()
    else:
        a.input_zero_point = int(zp)
    a.output_zero_point = int(zp_out)
    rx, ro = tk_gpu.ref(xd), tk_gpu.ref(out)
    tk_gpu._sync_check(lib.tk_requantize_fp(rx.ptr, ro.ptr, ctypes.byref(a), tk_gpu.stream()), "tk_requantize_fp")
    return out.cpu().numpy()


@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("case", load_cases("qnn.requantize"), ids=lambda c: f"{c['name']}-{c['attrs']['rounding']}")
def test_requantize_fp_kat(device, case, bits):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    if x.ndim == 0:
        x = x.reshape(1)
    got = requantize_fp_gpu(x, scale_const(a["input_scale"]), a["input_zero_point"], np.float32(a["output_scale"]),
                            a["output_zero_point"], a["axis"], a["rounding"], a["out_dtype"], bits)
    np.testing.assert_array_equal(got.reshape(-1), load_array(case["expected"]).reshape(-1))


@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("rounding", ["UPWARD", "TONEAREST"])
@pytest.mark.parametrize("in_dtype,out_dtype", [("int32", "int8"), ("int32", "uint8"), ("int32", "int32"),
                                                ("int8", "int8"), ("uint8", "int16")])
def test_requantize_fp_random(device, bits, rounding, in_dtype, out_dtype):
    rng = np.random.default_rng(17 + bits)
    info = np.iinfo(in_dtype)
    shape = (3, 37, 5, 7)
    x = rng.integers(info.min, int(info.max) + 1, size=shape, dtype=np.int64).astype(in_dtype)
    if in_dtype == "int32":  # small magnitudes too, where the rounding ties sit
        x.reshape(-1)[::3] = rng.integers(-300, 300, size=x.size // 3 + (x.size % 3 > 0))
    cd = f"float{bits}"
    cases = [
        (np.float32(0.0173), 3, np.float32(0.05), -4, 1),        # downscale, per-tensor
        (np.float32(0.25), 0, np.float32(0.25), 7, 1),           # equal scales: multiply skipped
        (np.float32(3.7), -2, np.float32(0.5), 1, 1),            # upscale: out-of-range products
        (rng.uniform(0.001, 2.0, size=37).astype(np.float32), rng.integers(-9, 9, size=37).astype(np.int32),
         np.float32(0.125), 5, 1),                               # per-axis scales and zero points
        (rng.uniform(0.5, 4.0, size=5).astype(np.float32), 0, np.float32(1.0), -1, 2),
    ]
    for s_in, zp_in, s_out, zp_out, axis in cases:
        if np.ndim(s_in) and s_in.size != shape[axis]:
            continue
        if np.ndim(zp_in) and np.size(zp_in) != shape[axis]:
            continue
        exp = ref.requantize(x, s_in, np.asarray(zp_in, np.int32), s_out, np.int32(zp_out), axis=axis,
                             rounding=rounding, out_dtype=out_dtype, compute_dtype=cd)
        got = requantize_fp_gpu(x, s_in, zp_in, s_out, zp_out, axis, rounding, out_dtype, bits)
        if not np.array_equal(got, exp):
            bad = np.argwhere(got != exp)[0]
            raise AssertionError(f"{cd} {rounding} s_in={s_in if np.ndim(s_in) == 0 else 'vec'}: first mismatch at "
                                 f"{tuple(bad)} x={x[tuple(bad)]}: gpu {got[tuple(bad)]} vs oracle {exp[tuple(bad)]}")


def test_float_forms_differ_from_int64(device):
    """The float32 form is not the int64 one in disguise: on large int32 inputs float32 rounds the
    data itself (24-bit significand), and the oracle and the device agree on the float32 answer."""
    x = np.array([16777217, 2147483000, -2147483000, 33554435, -16777219], dtype=np.int32)
    s_in, s_out = np.float32(1.0), np.float32(3.0)
    f32 = ref.requantize(x, s_in, np.int32(0), s_out, np.int32(0), out_dtype="int32", compute_dtype="float32")
    i64 = ref.requantize(x, s_in, np.int32(0), s_out, np.int32(0), out_dtype="int32")
    assert not np.array_equal(f32, i64)
    np.testing.assert_array_equal(requantize_fp_gpu(x, s_in, 0, s_out, 0, -1, "UPWARD", "int32", 32), f32)


def _trace(mod, params, inputs, tmp_path):
    lib = relay.build(mod, target="mi355x", params=params)
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input(**inputs)
    path = str(tmp_path / "t.tkt")
    m.dump_trace(path)
    return m, read_trace(path, copy=True).records


def _compare(records, expected):
    assert set(records) == set(expected)
    for name, e in expected.items():
        g = records[name]
        assert g.shape == e.shape and g.dtype == e.dtype, (name, g.shape, e.shape)
        if not np.array_equal(g, e):
            bad = np.argwhere(g != e)[0]
            raise AssertionError(f"record {name}: first mismatch at {tuple(bad)}: {g[tuple(bad)]} vs {e[tuple(bad)]}")


@pytest.mark.parametrize("cd", ["float32", "float64"])
@pytest.mark.parametrize("rounding", ["UPWARD", "TONEAREST"])
def test_lenet5_float_compute_trace(device, tmp_path, cd, rounding):
    """LeNet-5 built under requantize_config(compute_dtype=cd, rounding=...): every requantize runs
    as tk_requantize_fp (the conv / dense blocks unfused), every record bit-exact vs the oracle."""
    with qnn.op.requantize_config(rounding=rounding, compute_dtype=cd):
        model = zoo.lenet5(batch=2)
    x = model.random_input()
    m, rec = _trace(model.mod, model.params, {"data": x}, tmp_path)
    assert _lib.NODE_KINDS["requantize_fp"] in m.module.node_native_kinds
    _compare(rec, graph_ref.calibrate(model.mod, model.params, {"data": x}))


@pytest.mark.parametrize("cd", ["float32", "float64"])
def test_binary_ops_float_compute_trace(device, tmp_path, cd):
    """qnn.add (per-tensor and per-axis), qnn.subtract and qnn.mul (per-axis) built under a float
    compute_dtype: the inner requantizes in RequantizeLowerFP form on tk_qnn_binary_fp."""
    rng = np.random.default_rng(5)
    shape = (2, 8, 5, 6)
    a = relay.var("a", shape=shape, dtype="int8")
    b = relay.var("b", shape=shape, dtype="int8")
    sa = rng.uniform(0.01, 0.2, size=8).astype(np.float32)
    with qnn.op.requantize_config(compute_dtype=cd, rounding="TONEAREST"):
        add_t = qnn.op.add(a, b, relay.const(0.07, "float32"), relay.const(3, "int32"), relay.const(0.11, "float32"),
                           relay.const(-2, "int32"), relay.const(0.09, "float32"), relay.const(1, "int32"))
        add_c = qnn.op.add(add_t, b, relay.const(sa), relay.const(0, "int32"), relay.const(0.05, "float32"),
                           relay.const(4, "int32"), relay.const(0.13, "float32"), relay.const(-3, "int32"),
                           lhs_axis=1)
    with qnn.op.requantize_config(compute_dtype=cd):
        sub = qnn.op.subtract(add_c, a, relay.const(0.13, "float32"), relay.const(-3, "int32"),
                              relay.const(0.07, "float32"), relay.const(3, "int32"), relay.const(0.2, "float32"),
                              relay.const(0, "int32"))
        mul = qnn.op.mul(sub, b, relay.const(sa), relay.const(0, "int32"), relay.const(sa * 0.5), relay.const(1, "int32"),
                         relay.const(0.01, "float32"), relay.const(2, "int32"), lhs_axis=1, rhs_axis=1)
    mod = relay.IRModule.from_expr(mul)
    inputs = {"a": rng.integers(-128, 128, size=shape).astype(np.int8),
              "b": rng.integers(-128, 128, size=shape).astype(np.int8)}
    m, rec = _trace(mod, {}, inputs, tmp_path)
    assert m.module.node_native_kinds.count(_lib.NODE_KINDS["qnn_binary_fp"]) == 4
    _compare(rec, graph_ref.calibrate(mod, {}, inputs))

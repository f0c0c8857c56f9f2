"""Pin the CPU oracle (oracle/qnn_ref.py) to the reference's literal known-answer vectors."""
import numpy as np
import pytest

from oracle import qnn_ref as ref
from tests.golden_util import load_cases, load_array, scale_const


def _id(c):
    return f"{c['name']}-{c['attrs'].get('rounding', '')}"


# test_op_qnn_requantize.py:25 runs every case under the three compute dtypes against the same goldens
@pytest.mark.parametrize("compute_dtype", ["int64", "float32", "float64"])
@pytest.mark.parametrize("case", load_cases("qnn.requantize"), ids=_id)
def test_requantize_kat(case, compute_dtype):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    out = ref.requantize(x, scale_const(a["input_scale"]), np.int32(a["input_zero_point"]),
                         np.float32(a["output_scale"]), np.int32(a["output_zero_point"]),
                         axis=a["axis"], rounding=a["rounding"], out_dtype=a["out_dtype"],
                         compute_dtype=compute_dtype)
    np.testing.assert_array_equal(out, load_array(case["expected"]))
    assert out.dtype == np.dtype(a["out_dtype"])


@pytest.mark.parametrize("case", load_cases("qnn.dense"), ids=lambda c: c["name"])
def test_dense_kat(case):
    a = case["attrs"]
    out = ref.qnn_dense(load_array(case["inputs"]["data"]), load_array(case["inputs"]["weight"]),
                        a["input_zero_point"], a["kernel_zero_point"])
    if "bias" in case:
        out = ref.bias_add(out, load_array(case["bias"]), axis=1)
    if "requantize" in case:
        r = case["requantize"]
        out = ref.requantize(out, scale_const(r["input_scale"]), np.int32(0), np.float32(r["output_scale"]),
                             np.int32(r["output_zero_point"]), axis=-1, out_dtype=r["out_dtype"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.conv2d"), ids=lambda c: c["name"])
def test_conv2d_kat(case):
    a = case["attrs"]
    out = ref.qnn_conv2d(load_array(case["inputs"]["data"]), load_array(case["inputs"]["weight"]),
                         a["input_zero_point"], a["kernel_zero_point"], strides=a["strides"],
                         padding=a["padding"], dilation=a["dilation"], groups=a["groups"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.add"), ids=lambda c: c["name"])
def test_add_kat(case):
    a = case["attrs"]
    out = ref.qnn_add(load_array(case["inputs"]["lhs"]), load_array(case["inputs"]["rhs"]),
                      a["lhs_scale"], a["lhs_zero_point"], a["rhs_scale"], a["rhs_zero_point"],
                      a["output_scale"], a["output_zero_point"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


def test_fixed_point_multiplier_shift():
    # GetFixedPointMultiplierShift (src/relay/qnn/utils.cc:33-57)
    assert ref.get_fixed_point_multiplier_shift(0.0) == (0, 0)
    assert ref.get_fixed_point_multiplier_shift(1.0 / 16) == (1 << 30, -3)
    assert ref.get_fixed_point_multiplier_shift(1.0) == (1 << 30, 1)
    m, s = ref.get_fixed_point_multiplier_shift(1.0 / 3)
    assert s == -1 and m == round((2.0 / 3) * (1 << 31))
    # significand rounding up to 2^31 folds into 2^30 with exponent + 1
    m, s = ref.get_fixed_point_multiplier_shift(np.nextafter(1.0, 0.0))
    assert (m, s) == (1 << 30, 1)


def test_power_of_two_int32_path_wraps():
    # intrin_rule.cc:223-237 computes the rounding add in int32: INT32_MAX + 8 wraps negative
    x = np.array([2**31 - 1, 2**31 - 8, -2**31], dtype=np.int64)
    out = ref.q_multiply_shift(x, 1 << 30, -3)
    assert out[0] == ((2**31 - 1 + 8 - 2**32) >> 4)
    assert out[1] == ((2**31 - 8 + 8 - 2**32) >> 4)
    assert out[2] == ((-2**31 + 8) >> 4)


# ---- the pre-quantized QNN ops

def _p(v, dtype):
    return np.array(v, dtype=dtype) if isinstance(v, list) else np.dtype(dtype).type(v)


@pytest.mark.parametrize("case", load_cases("qnn.quantize"), ids=lambda c: c["name"])
def test_quantize_kat(case):
    a = case["attrs"]
    out = ref.quantize(load_array(case["inputs"]["data"]), _p(a["output_scale"], "float32"),
                       _p(a["output_zero_point"], "int32"), axis=a["axis"], out_dtype=a["out_dtype"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))
    assert out.dtype == np.dtype(a["out_dtype"])


@pytest.mark.parametrize("case", load_cases("qnn.dequantize"), ids=lambda c: c["name"])
def test_dequantize_kat(case):
    a = case["attrs"]
    out = ref.dequantize(load_array(case["inputs"]["data"]), _p(a["input_scale"], "float32"),
                         _p(a["input_zero_point"], "int32"), axis=a["axis"])
    exp = load_array(case["expected"])
    assert out.dtype == np.float32 and out.shape == exp.shape
    np.testing.assert_array_equal(out, exp)


@pytest.mark.parametrize("case", load_cases("qnn.concatenate"), ids=lambda c: c["name"])
def test_concatenate_kat(case):
    a = case["attrs"]
    out = ref.qnn_concatenate([load_array(d) for d in case["inputs"]["data"]],
                              [np.float32(s) for s in a["input_scales"]],
                              [np.int32(z) for z in a["input_zero_points"]], np.float32(a["output_scale"]),
                              np.int32(a["output_zero_point"]), axis=a["axis"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("op", ["qnn.mul", "qnn.subtract"])
def test_binary_kats(op):
    fn = ref.qnn_mul if op == "qnn.mul" else ref.qnn_subtract
    cases = load_cases(op)
    assert len(cases) == 9
    for case in cases:
        a = case["attrs"]
        out = fn(load_array(case["inputs"]["lhs"]), load_array(case["inputs"]["rhs"]), np.float32(a["lhs_scale"]),
                 np.int32(a["lhs_zero_point"]), np.float32(a["rhs_scale"]), np.int32(a["rhs_zero_point"]),
                 np.float32(a["output_scale"]), np.int32(a["output_zero_point"]))
        np.testing.assert_array_equal(out, load_array(case["expected"]), err_msg=case["name"])


def test_quantize_rounding_and_int32_edges():
    """llvm.round halves away from zero (0.5 -> 1, -0.5 -> -1, 2.5 -> 3), the division is one float32
    rounding, and an int32 output clips at float32(2^31 - 1) = 2^31, which x86's cvttss2si turns
    into INT32_MIN."""
    x = np.array([0.25, 0.5, -0.5, 1.25, 2.5, -2.5, 3e9, -3e9], np.float32)
    q = ref.quantize(x, np.float32(0.5), np.int32(0), out_dtype="int32")
    assert q.tolist() == [1, 1, -1, 3, 5, -5, -2 ** 31, -2 ** 31]
    # a value whose float32 quotient is not the float64 one: x / s rounded once in float32
    x = np.array([0.1], np.float32)
    s = np.float32(0.3)
    assert ref.quantize(x, s, np.int32(0), out_dtype="int8")[0] == int(np.round(np.float32(x[0] / s)))


def test_binary_broadcast_and_per_axis():
    """qnn.add / subtract / mul broadcast like numpy (BroadcastRel) and take per-axis parameters
    along each operand's axis (RequantizeOrUpcast / mul.cc per-channel branch)."""
    rng = np.random.default_rng(0)
    a = rng.integers(-128, 128, (2, 3, 4, 5)).astype(np.int8)
    b = rng.integers(-128, 128, (3, 1, 1)).astype(np.int8)
    out = ref.qnn_subtract(a, b, np.float32(0.02), np.int32(1), np.float32(0.03), np.int32(-2), np.float32(0.04),
                           np.int32(3))
    ra = ref.requantize(a, np.float32(0.02), np.int32(1), np.float32(0.04), np.int32(3), out_dtype="int32")
    rb = ref.requantize(b, np.float32(0.03), np.int32(-2), np.float32(0.04), np.int32(3), out_dtype="int32")
    exp = np.clip(ra.astype(np.int64) - rb + 3, -128, 127).astype(np.int8)
    np.testing.assert_array_equal(out, exp)
    # per-channel mul: scales along axis 1 of both operands
    ls = np.array([0.01, 0.02, 0.03], np.float32)
    rs = np.array([0.5, 0.25, 0.125], np.float32)
    c = rng.integers(-128, 128, (2, 3, 4, 5)).astype(np.int8)
    out = ref.qnn_mul(a, c, ls, np.int32(0), rs, np.int32(0), np.float32(0.05), np.int32(0), lhs_axis=1, rhs_axis=1)
    prod = a.astype(np.int64) * c
    sc = np.array([np.float32(np.float64(x) * np.float64(y)) for x, y in zip(ls, rs)], np.float32)
    exp = ref.requantize(prod, sc, np.int32(0), np.float32(0.05), np.int32(0), axis=1, out_dtype="int8")
    np.testing.assert_array_equal(out, exp)


# ---- round 5: the rest of the QNN dialect (leaky_relu, unary table lookups, batch_matmul,
# conv2d_transpose)

@pytest.mark.parametrize("case", load_cases("qnn.leaky_relu"), ids=lambda c: c["name"])
def test_leaky_relu_kat(case):
    a = case["attrs"]
    out = ref.qnn_leaky_relu(load_array(case["inputs"]["data"]), a["alpha"], a["input_scale"], a["input_zero_point"],
                             a["output_scale"], a["output_zero_point"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.unary"), ids=lambda c: c["name"])
def test_unary_kat(case):
    a = case["attrs"]
    out = ref.qnn_unary(a["unary_op"], load_array(case["inputs"]["data"]), a["scale"], a["zero_point"],
                        a["output_scale"], a["output_zero_point"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.batch_matmul"), ids=lambda c: c["name"])
def test_batch_matmul_kat(case):
    a = case["attrs"]
    out = ref.qnn_batch_matmul(load_array(case["inputs"]["x"]), load_array(case["inputs"]["y"]), a["x_zero_point"],
                               a["y_zero_point"])
    if "requantize" in case:
        r = case["requantize"]
        out = ref.requantize(out, np.float32(r["input_scale"]), np.int32(0), np.float32(r["output_scale"]),
                             np.int32(r["output_zero_point"]), out_dtype=r["out_dtype"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


def test_leaky_relu_alpha_one_is_rejected():
    # fixed_point_multiply by 1.0 takes q_multiply_shift's power-of-two branch with shift 1: the
    # reference's compiler rejects the 1 << -1 rounding factor (intrin_rule.cc:223-237)
    x = np.array([1, 2, 3], np.int8)
    with pytest.raises(ValueError):
        ref.qnn_leaky_relu(x, 1.0, 0.5, 0, 0.5, 0)
    with pytest.raises(ValueError):
        ref.qnn_leaky_relu(x, 0.0, 0.5, 0, 0.5, 0)


def _conv2d_transpose_topi(d, w, zd, zw, strides, padding, output_padding, groups):
    """The definition as topi writes it (conv2d_transpose.py:79-140): int16 shifts, dilate the data
    by the stride, pad by k - 1 - pad (+ output padding at the end), correlate with the kernel
    flipped and transposed to OIHW -- an independent restatement to pin qnn_ref's gather form."""
    d = d.astype(np.int64) - zd
    w = w.astype(np.int64) - (np.asarray(zw).reshape(1, -1, 1, 1) if np.ndim(zw) else zw)
    n, c, h, wd = d.shape
    _, og, kh, kw = w.shape
    sh, sw = strides
    pt, pl, pb, pr = padding
    dil = np.zeros((n, c, (h - 1) * sh + 1, (wd - 1) * sw + 1), np.int64)
    dil[:, :, ::sh, ::sw] = d
    pad = np.pad(dil, ((0, 0), (0, 0), (kh - 1 - pt, kh - 1 - pb + output_padding[0]),
                       (kw - 1 - pl, kw - 1 - pr + output_padding[1])))
    oh, ow = pad.shape[2] - kh + 1, pad.shape[3] - kw + 1
    cg = c // groups
    out = np.zeros((n, og * groups, oh, ow), np.int64)
    for o in range(og * groups):
        g, oo = divmod(o, og)
        kt = w[g * cg:(g + 1) * cg, oo, ::-1, ::-1]  # (cg, kh, kw), flipped
        for y in range(oh):
            for x in range(ow):
                out[:, o, y, x] = np.einsum("nchw,chw->n", pad[:, g * cg:(g + 1) * cg, y:y + kh, x:x + kw], kt)
    return ref.wrap_i32(out).astype(np.int32)


@pytest.mark.parametrize("cfg", [
    # test_op_qnn_conv2_transpose.py's shapes: no / kernel / input / both zero points, padding, strides
    ((2, 1, 2, 4), (1, 3, 2, 2), 0, 0, (1, 1), (0, 0, 0, 0), (0, 0), 1, "uint8"),
    ((2, 4, 2, 4), (4, 3, 2, 2), 0, 1, (1, 1), (0, 0, 0, 0), (0, 0), 1, "uint8"),
    ((2, 4, 2, 4), (4, 3, 2, 2), 5, 0, (1, 1), (0, 0, 0, 0), (0, 0), 1, "int8"),
    ((1, 4, 2, 2), (4, 3, 2, 2), 8, 5, (1, 1), (1, 1, 1, 1), (0, 0), 1, "uint8"),
    ((2, 4, 5, 3), (4, 2, 3, 3), 3, 2, (2, 2), (1, 0, 1, 2), (1, 1), 1, "int8"),
    ((1, 6, 4, 4), (6, 2, 3, 3), -2, 1, (2, 1), (0, 1, 1, 0), (1, 0), 3, "int8"),
    ((1, 4, 3, 3), (4, 3, 2, 2), 1, [1, -2, 3], (2, 2), (0, 0, 0, 0), (0, 0), 1, "uint8"),
])
def test_conv2d_transpose_oracle_matches_topi_definition(cfg):
    ds, ws, zd, zw, st, pad, opad, groups, dt = cfg
    rng = np.random.default_rng(7)
    info = np.iinfo(dt)
    d = rng.integers(info.min, info.max + 1, ds).astype(dt)
    w = rng.integers(info.min, info.max + 1, ws).astype(dt)
    got = ref.qnn_conv2d_transpose(d, w, zd, np.asarray(zw), strides=st, padding=pad, output_padding=opad,
                                   groups=groups)
    exp = _conv2d_transpose_topi(d, w, zd, zw, st, pad, opad, groups)
    np.testing.assert_array_equal(got, exp)


# ---------------------------------------------------------------- simulated (de)quantize
# test_op_qnn_simulated_{quantize,dequantize}.py hold no literals: each case checks that the
# simulated op equals qnn.quantize / qnn.dequantize on the same data and parameters (allowing 3
# mismatches for GPU float32).  The same cases, seeded, and the equality exact -- both sides are
# restated from the reference's float32 steps (quantize.cc:113-149 vs topi/nn/qnn.py:40-190).
SIM_CASES = [
    # (name, data range, shape, data dtype, scale, zero point, axis, dtype)
    ("simple_uint8", (-128, 127), (2, 5), "float32", 0.5, 127, -1, "uint8"),
    ("simple_int8", (-128, 127), (2, 5), "float32", 0.5, 127, -1, "int8"),
    ("simple_int32", (-128, 127), (2, 5), "float32", 0.5, 127, -1, "int32"),
    ("dynamic_channels_scalar", (-64, 64), (2, 5), "float32", [0.5], [127], 0, "uint8"),
    ("dynamic_channels_per_channel", (-64, 64), (2, 5), "float32", [0.5, 0.25], [127, 123], 0, "uint8"),
    ("dynamic_dtype_uint8", (-64, 64), (2, 5), "float32", [0.5], [127], -1, "uint8"),
    ("dynamic_dtype_int32", (-64, 64), (2, 5), "float32", [0.5], [127], -1, "int32"),
]


@pytest.mark.parametrize("case", SIM_CASES, ids=lambda c: c[0])
def test_simulated_quantize_equals_quantize(case):
    _, (lo, hi), shape, _, s, z, axis, dt = case
    x = np.random.default_rng(3).uniform(lo, hi, shape).astype(np.float32)
    x.reshape(-1)[:3] = [0.25, -0.75, 1e10]  # exact halves after / 0.5, past the int32 bound
    code = ref.SQNN_DTYPE_TO_CODE[dt]
    sim = ref.simulated_quantize(x, code, np.asarray(s, np.float32), np.asarray(z, np.int32), axis=axis)
    sv, zv = np.asarray(s, np.float32), np.asarray(z, np.int32)
    q = ref.quantize(x, sv if sv.size > 1 else sv.reshape(()), zv if zv.size > 1 else zv.reshape(()), axis=axis,
                     out_dtype=dt)
    if dt == "int32":
        # quantize's fptosi of the clipped 2^31 is INT32_MIN (x86 cvttss2si); the simulated op keeps
        # the float 2^31 -- the one place the two differ, where the reference test allows mismatches
        big = sim >= 2.0 ** 31
        assert big.sum() == 1 and q[big][0] == np.iinfo(np.int32).min
        q = np.where(big, np.float32(2.0 ** 31), q.astype(np.float32))
    np.testing.assert_array_equal(sim, q.astype(np.float32))


@pytest.mark.parametrize("case", [
    ("simple_uint8", (-128, 127), "uint8", 0.5, 127, -1),
    ("simple_int8", (-128, 127), "int8", 0.5, 127, -1),
    ("dynamic_channels_scalar", (-64, 64), "int8", [0.5], [0], 0),
    ("dynamic_channels_per_channel", (-64, 64), "int8", [0.5, 0.25], [127, 123], 0),
    ("dynamic_dtype_uint8", (0, 255), "uint8", [0.5], [127], -1),
    ("dynamic_dtype_int8", (0, 255), "int8", [0.5], [127], -1),
], ids=lambda c: c[0])
def test_simulated_dequantize_equals_dequantize(case):
    _, (lo, hi), dt, s, z, axis = case
    d = np.random.default_rng(4).uniform(lo, hi, (2, 5)).astype(dt)
    sim = ref.simulated_dequantize(d.astype(np.float32), ref.SQNN_DTYPE_TO_CODE[dt], np.asarray(s, np.float32),
                                   np.asarray(z, np.int32), axis=axis)
    sv, zv = np.asarray(s, np.float32), np.asarray(z, np.int32)
    dq = ref.dequantize(d, sv if sv.size > 1 else sv.reshape(()), zv if zv.size > 1 else zv.reshape(()), axis=axis)
    np.testing.assert_array_equal(sim, dq)


def test_simulated_ops_pass_through_and_modulo_indexing():
    x = np.array([[1.3, -2.5, 7.0, 300.0, -0.5]], np.float32)
    for code in (0, 4, -1):  # "disable" and any code outside the if_then_else chain
        np.testing.assert_array_equal(ref.simulated_quantize(x, code, [0.5], [1]), x)
        np.testing.assert_array_equal(ref.simulated_dequantize(x, code, [0.5], [1]), x)
    # 2 scales / 3 zero points on a 5-wide axis: element i takes scale[i % 2], zp[i % 3] (tir.indexmod)
    got = ref.simulated_quantize(x, 1, [0.5, 1.0], [0, 1, 2], axis=1)
    np.testing.assert_array_equal(got, np.array([[3.0, -2.0, 16.0, 127.0, 0.0]], np.float32))
    got = ref.simulated_dequantize(np.array([[4.0, 4.0, 4.0, 4.0, 4.0]], np.float32), 2, [0.5, 1.0], [0, 1, 2], axis=1)
    np.testing.assert_array_equal(got, np.array([[2.0, 3.0, 1.0, 4.0, 1.5]], np.float32))

"""Pin the CPU oracle (oracle/qnn_ref.py) to the reference's literal known-answer vectors."""
import numpy as np
import pytest

from oracle import qnn_ref as ref
from tests.golden_util import load_cases, load_array, scale_const


def _id(c):
    return f"{c['name']}-{c['attrs'].get('rounding', '')}"


@pytest.mark.parametrize("case", load_cases("qnn.requantize"), ids=_id)
def test_requantize_kat(case):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    out = ref.requantize(x, scale_const(a["input_scale"]), np.int32(a["input_zero_point"]),
                         np.float32(a["output_scale"]), np.int32(a["output_zero_point"]),
                         axis=a["axis"], rounding=a["rounding"], out_dtype=a["out_dtype"])
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

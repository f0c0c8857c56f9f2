"""Generate tests/golden/qnn_kats.json: the reference's literal known-answer vectors.

The reference (a TVM 0.11.dev0 fork) cannot be imported or built in this image
(``import tvm`` fails, submodules empty, no LLVM dev libs), so
these fixtures are *transcriptions of the literal input/expected-output data*
that the reference's own unit tests assert with ``np.testing.assert_equal`` on
target ``llvm``.  Each case records the test file:line it comes from.  Only
data (inputs, attributes, expected outputs) is stored — no reference source.

Run:  python tests/golden/make_golden.py   (rewrites qnn_kats.json)
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
RQ = "tests/python/relay/test_op_qnn_requantize.py"
DENSE = "tests/python/relay/test_op_qnn_dense.py"
CONV = "tests/python/relay/test_op_qnn_conv2d.py"
ADD = "tests/python/relay/test_op_qnn_add.py"
QUANT = "tests/python/relay/test_op_qnn_quantize.py"
DEQUANT = "tests/python/relay/test_op_qnn_dequantize.py"
CONCAT = "tests/python/relay/test_op_qnn_concatenate.py"
MUL = "tests/python/relay/test_op_qnn_mul.py"
SUB = "tests/python/relay/test_op_qnn_subtract.py"
LEAKY = "tests/python/relay/test_op_qnn_leaky_relu.py"
UNARY = "tests/python/relay/test_op_qnn_unary_elementwise.py"
BMM = "tests/python/relay/test_op_qnn_batch_matmul.py"


def arr(a, dtype):
    a = np.asarray(a).astype(dtype)
    flat = a.reshape(-1)
    if flat.size > 64 and np.all(flat == flat[0]):
        return {"dtype": dtype, "shape": list(a.shape), "fill": flat[0].item()}
    return {"dtype": dtype, "shape": list(a.shape), "data": flat.tolist()}


def rq_case(src, name, data, data_dtype, out_dtype, s_in, s_out, expect, rounding,
            zp_in=0, zp_out=0, axis=0, shape=None):
    d = np.asarray(data)
    if shape is not None:
        d = d.reshape(shape)
    e = np.asarray(expect).reshape(d.shape)
    return {
        "op": "qnn.requantize", "source": src, "name": name,
        "inputs": {"data": arr(d, data_dtype)},
        "attrs": {"input_scale": s_in, "input_zero_point": zp_in, "output_scale": s_out,
                  "output_zero_point": zp_out, "axis": axis, "rounding": rounding,
                  "out_dtype": out_dtype},
        "expected": arr(e, out_dtype),
    }


def requantize_cases():
    cases = []
    for rounding in ("UPWARD", "TONEAREST"):
        d = np.arange(-100, 100)
        cases.append(rq_case(f"{RQ}:81-98", "same_scale", d, "int32", "int8", 0.5, 0.5, d, rounding))
        cases.append(rq_case(f"{RQ}:101-117", "scalar_same_scale", np.array(-10), "int32", "int8",
                             0.5, 0.5, np.array(-10), rounding))
        # test_downscale (:120-204)
        pos = np.arange(0, 32)
        neg = np.arange(0, -32, -1)
        cases.append(rq_case(f"{RQ}:133-136", "downscale_16_pos", pos, "int32", "int8", 1.0, 16.0,
                             np.repeat([0, 1, 2], [8, 16, 8]), rounding))
        exp = np.repeat([0, -1, -2], [9, 16, 7]) if rounding == "UPWARD" else np.repeat([0, -1, -2], [8, 16, 8])
        cases.append(rq_case(f"{RQ}:138-144", "downscale_16_neg", neg, "int32", "int8", 1.0, 16.0, exp, rounding))
        cases.append(rq_case(f"{RQ}:156-160", "downscale_4_pos", pos, "int32", "int8", 1.0, 4.0,
                             np.repeat([0, 1, 2, 3, 4, 5, 6, 7, 8], [2, 4, 4, 4, 4, 4, 4, 4, 2]), rounding))
        if rounding == "UPWARD":
            exp = np.repeat([0, -1, -2, -3, -4, -5, -6, -7, -8], [3, 4, 4, 4, 4, 4, 4, 4, 1])
        else:
            exp = np.repeat([0, -1, -2, -3, -4, -5, -6, -7, -8], [2, 4, 4, 4, 4, 4, 4, 4, 2])
        cases.append(rq_case(f"{RQ}:162-173", "downscale_4_neg", neg, "int32", "int8", 1.0, 4.0, exp, rounding))
        cases.append(rq_case(f"{RQ}:175-189", "downscale_16_uint8_out", pos, "int32", "uint8", 1.0, 16.0,
                             np.repeat([0, 1, 2], [8, 16, 8]), rounding))
        cases.append(rq_case(f"{RQ}:191-204", "downscale_16_uint8_in_out", pos, "uint8", "uint8", 1.0, 16.0,
                             np.repeat([0, 1, 2], [8, 16, 8]), rounding))
        # test_upscale (:207-230)
        cases.append(rq_case(f"{RQ}:220-224", "upscale_pos", pos, "int32", "int8", 2.0, 1.0, 2 * pos, rounding))
        cases.append(rq_case(f"{RQ}:226-230", "upscale_neg", neg, "int32", "int8", 2.0, 1.0, 2 * neg, rounding))
        # test_non_power_of_two (:233-275)
        cases.append(rq_case(f"{RQ}:246-249", "npot_div3_pos", 3 * pos, "int32", "int8", 1.0, 3.0, pos, rounding))
        cases.append(rq_case(f"{RQ}:251-254", "npot_div3_neg", 3 * neg, "int32", "int8", 1.0, 3.0, neg, rounding))
        cases.append(rq_case(f"{RQ}:266-269", "npot_mul3_pos", pos, "int32", "int8", 3.0, 1.0, 3 * pos, rounding))
        cases.append(rq_case(f"{RQ}:271-274", "npot_mul3_neg", neg, "int32", "int8", 3.0, 1.0, 3 * neg, rounding))
        # test_saturation (:278-322)
        cases.append(rq_case(f"{RQ}:290-296", "saturation_pos", 120 + np.arange(16), "int32", "int8", 0.5, 0.5,
                             [120, 121, 122, 123, 124, 125, 126, 127] + [127] * 8, rounding))
        cases.append(rq_case(f"{RQ}:298-321", "saturation_neg", -120 - np.arange(16), "int32", "int8", 0.5, 0.5,
                             [-120, -121, -122, -123, -124, -125, -126, -127] + [-128] * 8, rounding))
        # test_zero_point (:325-384)
        cases.append(rq_case(f"{RQ}:340-344", "out_zp_pos", pos, "int32", "int8", 1.0, 16.0,
                             1 + np.repeat([0, 1, 2], [8, 16, 8]), rounding, zp_out=1))
        exp = np.repeat([-2, -3, -4], [9, 16, 7]) if rounding == "UPWARD" else np.repeat([-2, -3, -4], [8, 16, 8])
        cases.append(rq_case(f"{RQ}:346-353", "out_zp_neg", np.arange(-32, -64, -1), "int32", "int8", 1.0, 16.0,
                             1 + exp, rounding, zp_out=1))
        cases.append(rq_case(f"{RQ}:369-372", "in_zp_pos", np.arange(32, 64), "int32", "int8", 1.0, 16.0,
                             np.repeat([2, 3, 4], [8, 16, 8]) - 1, rounding, zp_in=16))
        cases.append(rq_case(f"{RQ}:374-381", "in_zp_neg", np.arange(-32, -64, -1), "int32", "int8", 1.0, 16.0,
                             exp - 1, rounding, zp_in=16))
        # per-channel (:387-479)
        d = np.arange(-5, 5).reshape(5, 2)
        cases.append(rq_case(f"{RQ}:389-403", "per_channel_same_scale_2d", d, "int32", "int8", [0.5, 0.5], 0.5,
                             d, rounding, axis=1))
        d = np.arange(-10, 10).reshape(2, 2, 5)
        cases.append(rq_case(f"{RQ}:405-420", "per_channel_same_scale_3d", d, "int32", "int8", [0.5, 0.5], 0.5,
                             d, rounding, axis=1))
        d = np.arange(-5, 5).reshape(5, 2)
        cases.append(rq_case(f"{RQ}:424-441", "per_channel_diff_scale_2d", d, "int32", "int8", [0.5, 0.25], 0.5,
                             [-5, -2, -3, -1, -1, 0, 1, 1, 3, 2], rounding, axis=1))
        d = np.arange(-20, 20, 2).reshape(2, 2, 5)
        cases.append(rq_case(f"{RQ}:443-460", "per_channel_diff_scale_3d", d, "int32", "int8", [0.5, 0.25], 0.5,
                             [-20, -18, -16, -14, -12, -5, -4, -3, -2, -1, 0, 2, 4, 6, 8, 5, 6, 7, 8, 9],
                             rounding, axis=1))
        d = np.arange(-5, 5).reshape(5, 2)
        cases.append(rq_case(f"{RQ}:462-479", "per_channel_in_gt_out_2d", d, "int32", "int8", [1.0, 0.25], 0.5,
                             [-10, -2, -6, -1, -2, 0, 2, 1, 6, 2], rounding, axis=1))
    # test_default_cfg_and_no_args (:482-492): default rounding is UPWARD
    cases.append(rq_case(f"{RQ}:482-492", "default_cfg", np.arange(0, -32, -1), "int32", "int8", 1.0, 16.0,
                         np.repeat([0, -1, -2], [9, 16, 7]), "UPWARD"))
    return cases


def dense_cases():
    data = np.array([1, 3, 5, 7, 9, 11, 13, 15, -19, -21, 1, 3, 5, 7, 9, 11, 13, -17, 17, -21]).reshape(2, 10)
    kernel = np.tile(np.array([1, 3, 5, 7, 9, 11, 13, 15, 17, 19]), 3).reshape(3, 10)
    base = {"op": "qnn.dense", "inputs": {"data": arr(data, "int8"), "weight": arr(kernel, "int8")},
            "attrs": {"input_zero_point": -1, "kernel_zero_point": -1, "input_scale": 0.5,
                      "kernel_scale": 0.5, "units": 3}}
    cases = []
    c = json.loads(json.dumps(base))
    c.update(source=f"{DENSE}:81-145,223-228", name="dense_no_bias",
             expected=arr(np.array([92, 92, 92, 228, 228, 228]).reshape(2, 3), "int32"))
    cases.append(c)
    c = json.loads(json.dumps(base))
    c.update(source=f"{DENSE}:81-145,231-236", name="dense_bias", bias=arr([4, 8, 12], "int32"),
             expected=arr(np.array([96, 100, 104, 232, 236, 240]).reshape(2, 3), "int32"))
    cases.append(c)
    c = json.loads(json.dumps(base))
    c.update(source=f"{DENSE}:81-145,239-245", name="dense_bias_requantize", bias=arr([4, 8, 12], "int32"),
             requantize={"input_scale": 0.25, "output_scale": 1.0, "output_zero_point": -1, "out_dtype": "int8"},
             expected=arr(np.array([23, 24, 25, 57, 58, 59]).reshape(2, 3), "int8"))
    cases.append(c)
    # per-channel: requantize input_scale = 0.5 * float32([0.5, 0.3, 0.4]) computed in float32
    pc = (0.5 * np.array([0.5, 0.3, 0.4], dtype=np.float32)).astype(np.float32)
    c = json.loads(json.dumps(base))
    c.update(source=f"{DENSE}:131-133,248-252", name="dense_per_channel", bias=arr([4, 8, 12], "int32"),
             requantize={"input_scale": [float(v) for v in pc], "output_scale": 1.0, "output_zero_point": -1,
                         "out_dtype": "int8"},
             expected=arr(np.array([23, 14, 20, 57, 34, 47]).reshape(2, 3), "int8"))
    cases.append(c)
    return cases


def conv_cases():
    cases = []
    cases.append({
        "op": "qnn.conv2d", "source": f"{CONV}:766-803", "name": "tflite_large_irregular",
        "inputs": {"data": arr(np.full((1, 1024, 1, 1), 127), "uint8"),
                   "weight": arr(np.full((1001, 1024, 1, 1), 127), "uint8")},
        "attrs": {"input_zero_point": 127, "kernel_zero_point": 127, "strides": [1, 1], "padding": [0, 0, 0, 0],
                  "dilation": [1, 1], "groups": 1},
        "expected": arr(np.zeros((1, 1001, 1, 1)), "int32"),
    })
    data = 128 + np.array((1, 1, 1, 1, 2, 2, 2, 2, 1, 2, 3, 4, 1, 2, 3, 4)).reshape(2, 1, 2, 4)
    weight = 128 + np.array((1, 2, 3, 4, -1, 1, -1, 1, -1, -1, 1, 1)).reshape(3, 1, 2, 2)
    cases.append({
        "op": "qnn.conv2d", "source": f"{CONV}:806-848", "name": "tflite_output_multiplier_greater_than_one",
        "inputs": {"data": arr(data, "uint8"), "weight": arr(weight, "uint8")},
        "attrs": {"input_zero_point": 128, "kernel_zero_point": 128, "strides": [2, 2], "padding": [0, 0, 0, 0],
                  "dilation": [1, 1], "groups": 1},
        "expected": arr(np.array((17, 17, 0, 0, 2, 2, 16, 36, 2, 2, 0, 0)).reshape(2, 3, 1, 2), "int32"),
    })
    data = np.array((133, 131, 129, 125, 123, 121, 135, 133, 131, 123, 121, 119, 137, 135, 133, 121, 119,
                     117)).reshape(1, 1, 3, 6)
    weight = np.array((129, 131, 133, 135)).reshape(1, 1, 2, 2)
    cases.append({
        "op": "qnn.conv2d", "source": f"{CONV}:851-911", "name": "tflite_anisotropic_strides",
        "inputs": {"data": arr(data, "uint8"), "weight": arr(weight, "uint8")},
        "attrs": {"input_zero_point": 127, "kernel_zero_point": 127, "strides": [1, 3], "padding": [0, 0, 0, 0],
                  "dilation": [1, 1], "groups": 1},
        "expected": arr(np.array((124, -92, 164, -132)).reshape(1, 1, 2, 2), "int32"),
    })
    return cases


def add_case(src, name, x, y, ls, lz, rs, rz, os_, oz, expect):
    return {"op": "qnn.add", "source": src, "name": name,
            "inputs": {"lhs": arr(np.array(x).reshape(1, 4), "uint8"), "rhs": arr(np.array(y).reshape(1, 4), "uint8")},
            "attrs": {"lhs_scale": ls, "lhs_zero_point": lz, "rhs_scale": rs, "rhs_zero_point": rz,
                      "output_scale": os_, "output_zero_point": oz},
            "expected": arr(np.array(expect).reshape(1, 4), "uint8")}


def add_cases():
    c = []
    xs = [(140, 153, 165, 178), (25, 153, 178, 216), (25, 153, 216, 165)]
    ys = [(204, 178, 165, 140), (204, 178, 191, 25), (204, 178, 25, 191)]
    gs = [(217, 204, 203, 191), (102, 204, 242, 114), (102, 204, 114, 229)]
    for i in range(3):
        c.append(add_case(f"{ADD}:23-69", f"same_io_params_{i}", xs[i], ys[i], 0.00784314, 127, 0.00784314, 127,
                          0.00784314, 127, gs[i]))
    xs = [(76, 140, 153, 172), (133, 140, 146, 153), (76, 140, 172, 146)]
    ys = [(136, 119, 128, 17), (136, 119, 111, 94), (136, 119, 17, 128)]
    gs = [(120, 154, 167, 124), (158, 154, 154, 150), (120, 154, 124, 163)]
    for i in range(3):
        c.append(add_case(f"{ADD}:72-118", f"different_io_params_{i}", xs[i], ys[i], 0.0156863, 127, 0.0117647, 85,
                          0.0235294, 128, gs[i]))
    c.append(add_case(f"{ADD}:121-150", "saturation_same", (255, 1, 1, 0), (255, 255, 128, 0), 0.125, 0, 0.125, 0,
                      0.125, 0, (255, 255, 129, 0)))
    c.append(add_case(f"{ADD}:152-177", "saturation_out_scale", (255, 1, 1, 0), (255, 255, 127, 0), 0.125, 0, 0.125,
                      0, 0.25, 0, (255, 129, 65, 0)))
    c.append(add_case(f"{ADD}:205-232", "saturation_all_diff", (255, 0, 1, 0), (0, 128, 64, 0), 0.5, 0, 0.25, 0,
                      0.125, 0, (255, 255, 132, 0)))
    return c


def quantize_cases():
    """test_op_qnn_quantize.py: literal float32 inputs and their int8 / uint8 codes."""
    c = []
    d = np.array([-63.5, -63, -62.5, -62, -61.5, 62, 62.5, 63, 63.5, 64], dtype="float32").reshape(2, 5)
    for name, src, zp, out_dtype, exp in (
            ("float32_to_uint8", f"{QUANT}:51-66", 127, "uint8", [0, 1, 2, 3, 4, 251, 252, 253, 254, 255]),
            ("float32_to_int8", f"{QUANT}:69-88", -1, "int8", [-128, -127, -126, -125, -124, 123, 124, 125, 126, 127])):
        c.append({"op": "qnn.quantize", "source": src, "name": name, "inputs": {"data": arr(d, "float32")},
                  "attrs": {"output_scale": 0.5, "output_zero_point": zp, "axis": -1, "out_dtype": out_dtype},
                  "expected": arr(np.array(exp).reshape(2, 5), out_dtype)})
    c.append({"op": "qnn.quantize", "source": f"{QUANT}:91-102", "name": "scalar_float32_to_int8",
              "inputs": {"data": arr(np.array(-63.5), "float32")},
              "attrs": {"output_scale": 0.5, "output_zero_point": -1, "axis": -1, "out_dtype": "int8"},
              "expected": arr(np.array(-128), "int8")})
    d = np.array([-63.5, -63, -62.5, -62, -61.5, 30, 31, 31.5, 31.75, 32], dtype="float32").reshape(2, 5)
    e = np.array([0, 1, 2, 3, 4, 243, 247, 249, 250, 251]).reshape(2, 5)
    c.append({"op": "qnn.quantize", "source": f"{QUANT}:105-124", "name": "channelwise_axis_0",
              "inputs": {"data": arr(d, "float32")},
              "attrs": {"output_scale": [0.5, 0.25], "output_zero_point": [127, 123], "axis": 0, "out_dtype": "uint8"},
              "expected": arr(e, "uint8")})
    c.append({"op": "qnn.quantize", "source": f"{QUANT}:127-148", "name": "channelwise_axis_1",
              "inputs": {"data": arr(d.T, "float32")},
              "attrs": {"output_scale": [0.5, 0.25], "output_zero_point": [127, 123], "axis": -1,
                        "out_dtype": "uint8"},
              "expected": arr(e.T, "uint8")})
    return c


def dequantize_cases():
    """test_op_qnn_dequantize.py: literal codes and their float32 values."""
    c = []
    f = np.array([-63.5, -63, -62.5, -62, -61.5, 62, 62.5, 63, 63.5, 64], dtype="float32")
    c.append({"op": "qnn.dequantize", "source": f"{DEQUANT}:47-57", "name": "uint8_to_float32",
              "inputs": {"data": arr(np.array([0, 1, 2, 3, 4, 251, 252, 253, 254, 255]).reshape(2, 5), "uint8")},
              "attrs": {"input_scale": 0.5, "input_zero_point": 127, "axis": -1},
              "expected": arr(f.reshape(2, 5), "float32")})
    c.append({"op": "qnn.dequantize", "source": f"{DEQUANT}:60-74", "name": "int8_to_float32",
              "inputs": {"data": arr(np.array([-128, -127, -126, -125, -124, 123, 124, 125, 126, 127]).reshape(2, 5),
                                     "int8")},
              "attrs": {"input_scale": 0.5, "input_zero_point": -1, "axis": -1},
              "expected": arr(f.reshape(2, 5), "float32")})
    c.append({"op": "qnn.dequantize", "source": f"{DEQUANT}:77-83", "name": "scalar_int8_to_float32",
              "inputs": {"data": arr(np.array(-128), "int8")},
              "attrs": {"input_scale": 0.5, "input_zero_point": -1, "axis": -1},
              "expected": arr(np.array(-63.5), "float32")})
    c.append({"op": "qnn.dequantize", "source": f"{DEQUANT}:86-92", "name": "int32_to_float32",
              "inputs": {"data": arr(np.array([113, 29, -1052]), "int32")},
              "attrs": {"input_scale": 0.0057968604, "input_zero_point": 0, "axis": -1},
              "expected": arr(np.array([0.6550452, 0.16810896, -6.098297]), "float32")})
    codes = np.array([0, 1, 2, 3, 4, 243, 247, 249, 250, 251]).reshape(2, 5)
    vals = np.array([-63.5, -63, -62.5, -62, -61.5, 30, 31, 31.5, 31.75, 32]).reshape(2, 5)
    c.append({"op": "qnn.dequantize", "source": f"{DEQUANT}:95-111", "name": "channelwise_axis_1",
              "inputs": {"data": arr(codes.T, "uint8")},
              "attrs": {"input_scale": [0.5, 0.25], "input_zero_point": [127, 123], "axis": -1},
              "expected": arr(vals.T, "float32")})
    c.append({"op": "qnn.dequantize", "source": f"{DEQUANT}:114-128", "name": "channelwise_axis_0",
              "inputs": {"data": arr(codes, "uint8")},
              "attrs": {"input_scale": [0.5, 0.25], "input_zero_point": [127, 123], "axis": 0},
              "expected": arr(vals, "float32")})
    c.append({"op": "qnn.dequantize", "source": f"{DEQUANT}:131-142", "name": "per_tensor_vector_args",
              "inputs": {"data": arr(np.array([0, 1, 2, 3, 4, 251, 252, 253, 254, 255]), "uint8")},
              "attrs": {"input_scale": [0.5], "input_zero_point": [127], "axis": -1},
              "expected": arr(f, "float32")})
    return c


def concatenate_cases():
    """test_op_qnn_concatenate.py: int32 ramps; the goldens are the test's own expressions."""
    c = []
    x = np.arange(-32, 32, 1).reshape(1, 64)
    y = np.arange(-64, 64, 2).reshape(1, 64)
    s = float(np.float32((62 + 64) / (np.power(2, 32) - 1.0)))
    for name, src, zps, ozp, gold in (
            ("same_io_qnn_params", f"{CONCAT}:26-57", (0, 0), 0, np.concatenate((x, y), axis=0)),
            ("different_io_qnn_params", f"{CONCAT}:60-93", (3, 4), 1, np.concatenate((x - 2, y - 3), axis=0)),
            ("few_same_io_qnn_params", f"{CONCAT}:96-129", (0, 1), 1, np.concatenate((x + 1, y), axis=0)),
            ("same_i_qnn_params", f"{CONCAT}:132-165", (0, 0), 1, np.concatenate((x + 1, y + 1), axis=0))):
        c.append({"op": "qnn.concatenate", "source": src, "name": name,
                  "inputs": {"data": [arr(x, "int32"), arr(y, "int32")]},
                  "attrs": {"input_scales": [s, s], "input_zero_points": list(zps), "output_scale": s,
                            "output_zero_point": ozp, "axis": 0},
                  "expected": arr(gold, "int32")})
    # test_call_input (:168-191): the two halves of a uint8 split, same params -> the input back
    ones = np.ones(64, dtype="uint8")
    c.append({"op": "qnn.concatenate", "source": f"{CONCAT}:168-191", "name": "call_input_split_halves",
              "inputs": {"data": [arr(ones[:32], "uint8"), arr(ones[32:], "uint8")]},
              "attrs": {"input_scales": [1.0, 1.0], "input_zero_points": [0, 0], "output_scale": 1.0,
                        "output_zero_point": 0, "axis": 0},
              "expected": arr(ones, "uint8")})
    return c


def _binary_case(op, src, name, x, y, ls, lz, rs, rz, os_, oz, expect):
    return {"op": op, "source": src, "name": name,
            "inputs": {"lhs": arr(np.array(x).reshape(1, 4), "uint8"), "rhs": arr(np.array(y).reshape(1, 4), "uint8")},
            "attrs": {"lhs_scale": ls, "lhs_zero_point": lz, "rhs_scale": rs, "rhs_zero_point": rz,
                      "output_scale": os_, "output_zero_point": oz},
            "expected": arr(np.array(expect).reshape(1, 4), "uint8")}


def mul_cases():
    """test_op_qnn_mul.py: the test's golden is its own float64 expression (recover both operands,
    multiply, np.around(v / s_out + zp_out), clip to uint8), evaluated here on its literal data."""
    def golden(x, y, ls, lz, rs, rz, os_, oz):
        xr = ls * (np.asarray(x) - lz)
        yr = rs * (np.asarray(y) - rz)
        return np.clip(np.around(xr * yr / os_ + oz), 0, 255).astype("uint8")

    c = []
    groups = [
        (f"{MUL}:39-87", "same_io_qnn_params", (0.00784314, 127, 0.00784314, 127, 0.00784314, 127),
         [(1, 153, 2, 178), (25, 1, 178, 216), (25, 153, 1, 165)],
         [(204, 178, 1, 8), (204, 178, 191, 1), (204, 178, 1, 191)]),
        (f"{MUL}:90-141", "different_io_qnn_params", (0.0156863, 127, 0.0117647, 85, 0.0235294, 128),
         [(76, 140, 153, 172), (133, 140, 146, 153), (76, 140, 172, 146)],
         [(136, 119, 128, 17), (136, 119, 111, 94), (136, 119, 17, 128)]),
        (f"{MUL}:144-180", "saturation_same", (0.125, 0, 0.125, 0, 0.125, 0), [(255, 1, 1, 0)], [(255, 255, 128, 0)]),
        (f"{MUL}:182-215", "saturation_out_scale", (0.125, 0, 0.125, 0, 0.25, 0), [(255, 1, 1, 0)],
         [(255, 255, 127, 0)]),
        (f"{MUL}:217-251", "saturation_all_diff", (0.5, 0, 0.25, 0, 0.125, 0), [(255, 0, 1, 0)], [(0, 128, 64, 0)]),
    ]
    for src, name, p, xs, ys in groups:
        for i, (x, y) in enumerate(zip(xs, ys)):
            c.append(_binary_case("qnn.mul", src, f"{name}_{i}", x, y, *p, golden(x, y, *p)))
    return c


def subtract_cases():
    """test_op_qnn_subtract.py: literal operands and goldens."""
    c = []
    groups = [
        (f"{SUB}:61-85", "same_io_qnn_params", (0.00784314, 127, 0.00784314, 127, 0.00784314, 127),
         [(140, 153, 165, 178), (25, 153, 178, 216), (25, 153, 216, 165)],
         [(204, 178, 165, 140), (204, 178, 191, 25), (204, 178, 25, 191)],
         [(63, 102, 127, 165), (0, 102, 114, 255), (0, 102, 255, 101)]),
        (f"{SUB}:88-112", "different_io_qnn_params", (0.0156863, 127, 0.0117647, 85, 0.0235294, 128),
         [(76, 140, 153, 172), (133, 140, 146, 153), (76, 140, 172, 146)],
         [(136, 119, 128, 17), (136, 119, 111, 94), (136, 119, 17, 128)],
         [(68, 120, 123, 192), (106, 120, 128, 140), (68, 120, 192, 119)]),
        (f"{SUB}:115-128", "saturation_same", (0.125, 0, 0.125, 0, 0.125, 0), [(255, 1, 1, 0)], [(255, 255, 128, 0)],
         [(0, 0, 0, 0)]),
        (f"{SUB}:130-142", "saturation_out_scale", (0.125, 0, 0.125, 0, 0.25, 0), [(255, 1, 200, 0)],
         [(255, 255, 127, 0)], [(0, 0, 36, 0)]),
        (f"{SUB}:144-156", "saturation_all_diff", (0.5, 0, 0.25, 0, 0.125, 0), [(255, 0, 1, 0)], [(0, 128, 64, 0)],
         [(255, 0, 0, 0)]),
    ]
    for src, name, p, xs, ys, gs in groups:
        for i, (x, y, g) in enumerate(zip(xs, ys, gs)):
            c.append(_binary_case("qnn.subtract", src, f"{name}_{i}", x, y, *p, g))
    return c


def leaky_relu_cases():
    """test_op_qnn_leaky_relu.py:36-73: the test's own golden formula (dequantize, alpha, np.around,
    clip to uint8) on its literal data."""
    x = np.array((255, 133, 0, 9)).reshape((1, 4))
    s_in, z_in, s_out, z_out, alpha = 0.125, 60, 0.6, 17, 0.9
    deq = s_in * (x - z_in)
    prod = np.clip(np.around(deq * alpha / s_out + z_out), 0, 255)
    rq = np.clip(np.round(deq / s_out + z_out), 0, 255)
    gold = np.where(x < z_in, prod, rq)
    return [{"op": "qnn.leaky_relu", "source": f"{LEAKY}:24-73", "name": "qnn_leaky_relu",
             "inputs": {"data": arr(x, "uint8")},
             "attrs": {"alpha": alpha, "input_scale": s_in, "input_zero_point": z_in, "output_scale": s_out,
                       "output_zero_point": z_out},
             "expected": arr(gold, "uint8")}]


def unary_cases():
    """test_op_qnn_unary_elementwise.py: golden = np.around(f(scale * (x - zp)) / s_out + zp_out), clipped,
    the float function evaluated in float64 on the test's literal inputs (every bit pattern, or
    the rsqrt saturation vector).  `class Sqrt` lacks the Test prefix (not collected there)."""
    import scipy.special

    def hardswish(x):
        x2 = np.clip(x + 3.0, 0.0, 6.0)
        return x * x2 / 6.0

    fns = {"qnn.rsqrt": lambda x: 1 / np.sqrt(x), "qnn.exp": np.exp, "qnn.tanh": np.tanh,
           "qnn.erf": scipy.special.erf, "qnn.sigmoid": lambda x: 1 / (1 + np.exp(-x)), "qnn.hardswish": hardswish}
    lines = {"qnn.rsqrt": "129-165", "qnn.exp": "181-186", "qnn.tanh": "189-194", "qnn.erf": "197-202",
             "qnn.sigmoid": "205-210", "qnn.hardswish": "213-218"}

    def gold(op, x, s, z, os_, oz, dt):
        with np.errstate(all="ignore"):
            o = fns[op](s * (np.asarray(x, dtype=np.float64) - z))
        o = np.around(o / os_ + oz)
        info = np.iinfo(dt)
        return np.clip(o, info.min, info.max).astype(dt)

    def case(op, name, x, dt, s, z, os_, oz):
        return {"op": "qnn.unary", "source": f"{UNARY}:{lines[op]}", "name": f"{op.split('.')[1]}_{name}",
                "inputs": {"data": arr(x, dt)},
                "attrs": {"unary_op": op, "scale": s, "zero_point": z, "output_scale": os_, "output_zero_point": oz},
                "expected": arr(gold(op, x, s, z, os_, oz, dt), dt)}

    c = []
    sat = np.array((255, 133, 0, 9)).reshape((1, 4))
    c.append(case("qnn.rsqrt", "saturation_same", sat, "uint8", 0.125, 0, 0.125, 0))
    c.append(case("qnn.rsqrt", "saturation_out_scale", sat, "uint8", 0.125, 0, 0.25, 0))
    for op in fns:
        c.append(case(op, "all_uint8", np.arange(0, 256, dtype="uint8"), "uint8", 0.125, 0, 0.125, 0))
        x8 = np.arange(1, 128, dtype="int8") if op == "qnn.rsqrt" else np.arange(0, 256, dtype="uint8").view("int8")
        c.append(case(op, "all_int8", x8, "int8", 0.125, 0, 0.125, 0))
    return c


def batch_matmul_cases():
    """test_op_qnn_batch_matmul.py:78-174: literal operands and outputs for batch sizes 1, 4, 7 and
    the four zero-point combinations, plus the requantized int8 output."""
    xv = [1, 3, 5, 7, 9, 11, 13, 15, -19, -21, 1, 3, 5, 7, 9, 11, 13, -17, 17, -21]
    yv = [1, 3, 5, 7, 9, 11, 13, 15, 17, 19, 1, 3, 5, 7, 9]
    outs = {(True, True): [165, 415, 165, -197, -207, -197, 165, 415, 165, -105, -75, -105],
            (False, False): [81960, 88360, 81960, 78400, 84540, 78400, 81960, 88360, 81960, 78984, 85164, 78984],
            (True, False): [3240, 3490, 3240, -320, -330, -320, 3240, 3490, 3240, 264, 294, 264],
            (False, True): [3240, 9640, 3240, 2878, 9018, 2878, 3240, 9640, 3240, 2970, 9150, 2970]}
    c = []
    for b in (1, 4, 7):
        x = np.array(xv)[np.newaxis, np.newaxis, :].repeat(b, axis=1).astype("int8").reshape(b, 4, 5)
        y = np.array(yv)[np.newaxis, np.newaxis, :].repeat(b, axis=1).astype("int8").reshape(b, 3, 5)
        for (xz0, yz0), o in outs.items():
            exp = np.array(o)[np.newaxis, np.newaxis, :].repeat(b, axis=1).reshape(b, 4, 3)
            c.append({"op": "qnn.batch_matmul", "source": f"{BMM}:73-174", "name": f"b{b}_xzp{int(not xz0)}_yzp{int(not yz0)}",
                      "inputs": {"x": arr(x, "int8"), "y": arr(y, "int8")},
                      "attrs": {"x_zero_point": 0 if xz0 else -123, "y_zero_point": 0 if yz0 else -123,
                                "x_scale": 0.5, "y_scale": 0.5},
                      "expected": arr(exp, "int32")})
        exp = np.array([20, 51, 20, -26, -27, -26, 20, 51, 20, -14, -10, -14])[np.newaxis, np.newaxis, :].repeat(
            b, axis=1).reshape(b, 4, 3)
        c.append({"op": "qnn.batch_matmul", "source": f"{BMM}:131-158,259-265", "name": f"b{b}_requantized",
                  "inputs": {"x": arr(x, "int8"), "y": arr(y, "int8")},
                  "attrs": {"x_zero_point": 0, "y_zero_point": 0, "x_scale": 0.5, "y_scale": 0.5},
                  "requantize": {"input_scale": 0.25, "output_scale": 2.0, "output_zero_point": -1, "out_dtype": "int8"},
                  "expected": arr(exp, "int8")})
    return c


def main():
    doc = {
        "about": "Literal known-answer vectors transcribed from the reference's unit tests "
                 "(CortexFoundation/tachikoma @ /root/reference). Generated by make_golden.py.",
        "pinned_config": {"target": "llvm (no -mcpu)", "compute_dtype": "int64", "rounding_default": "UPWARD"},
        "cases": requantize_cases() + dense_cases() + conv_cases() + add_cases() + quantize_cases() +
                 dequantize_cases() + concatenate_cases() + mul_cases() + subtract_cases() + leaky_relu_cases() +
                 unary_cases() + batch_matmul_cases(),
    }
    path = os.path.join(HERE, "qnn_kats.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=None, separators=(",", ":"))
    print(f"wrote {len(doc['cases'])} cases to {path}")


if __name__ == "__main__":
    main()

"""Per-op parity through the C ABI on the MI355X vs the CPU oracle (bit-exact).

Covers the reference's literal KATs (tests/golden/qnn_kats.json) and seeded random
sweeps over the edge cases the reference tests: zero points (scalar / per-channel),
uint8 operands, strides, padding, dilation, groups/depthwise, ragged K and M,
saturation, per-axis requantize, both rounding modes.
"""
import zlib

import numpy as np
import pytest

from oracle import qnn_ref as ref
from tests.golden_util import load_array, load_cases, scale_const

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tk(device):
    from tests import tk_gpu
    return tk_gpu


@pytest.mark.parametrize("case", load_cases("qnn.requantize"), ids=lambda c: f"{c['name']}-{c['attrs']['rounding']}")
def test_requantize_kat(tk, case):
    a = case["attrs"]
    x = load_array(case["inputs"]["data"])
    out = tk.requantize(x, scale_const(a["input_scale"]), np.int32(a["input_zero_point"]), np.float32(a["output_scale"]),
                        a["output_zero_point"], axis=a["axis"], rounding=a["rounding"], out_dtype=a["out_dtype"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.dense"), ids=lambda c: c["name"])
def test_dense_kat(tk, case):
    a = case["attrs"]
    out = tk.dense(load_array(case["inputs"]["data"]), load_array(case["inputs"]["weight"]), a["input_zero_point"],
                   a["kernel_zero_point"])
    if "bias" in case:
        out = tk.bias_add(out, load_array(case["bias"]), axis=1)
    if "requantize" in case:
        r = case["requantize"]
        out = tk.requantize(out, scale_const(r["input_scale"]), np.int32(0), np.float32(r["output_scale"]),
                            r["output_zero_point"], axis=-1, out_dtype=r["out_dtype"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.conv2d"), ids=lambda c: c["name"])
def test_conv2d_kat(tk, case):
    a = case["attrs"]
    out = tk.conv2d(load_array(case["inputs"]["data"]), load_array(case["inputs"]["weight"]), a["input_zero_point"],
                    a["kernel_zero_point"], strides=a["strides"], padding=a["padding"], dilation=a["dilation"],
                    groups=a["groups"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


@pytest.mark.parametrize("case", load_cases("qnn.add"), ids=lambda c: c["name"])
def test_add_kat(tk, case):
    a = case["attrs"]
    out = tk.qnn_add(load_array(case["inputs"]["lhs"]), load_array(case["inputs"]["rhs"]), a["lhs_scale"],
                     a["lhs_zero_point"], a["rhs_scale"], a["rhs_zero_point"], a["output_scale"],
                     a["output_zero_point"])
    np.testing.assert_array_equal(out, load_array(case["expected"]))


def blocked_shadow(x: np.ndarray) -> np.ndarray:
    """Expected tk_conv2d_make_shadow layout of an NCHW 8-bit tensor: [C_pad16/16][N*H*W][16] uint8,
    padded channels 0, uint8 stored xor 0x80."""
    n, c, h, w = x.shape
    cpad = (c + 15) // 16 * 16
    b = x.view(np.uint8) ^ (0x80 if x.dtype == np.uint8 else 0)
    full = np.zeros((n, cpad, h, w), np.uint8)
    full[:, :c] = b
    return full.reshape(n, cpad // 16, 16, h * w).transpose(1, 0, 3, 2).reshape(cpad // 16, n * h * w, 16)


def _rand(rng, shape, dtype):
    info = np.iinfo(dtype)
    return rng.integers(info.min, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


CONV_CASES = [
    # (N, C, H, W, O, K, stride, pad, dilation, groups, dtype_x, dtype_w, za, zw)
    (2, 16, 9, 9, 32, 3, 1, 1, 1, 1, "int8", "int8", -3, 0),
    (1, 3, 17, 19, 64, 7, 2, 3, 1, 1, "int8", "int8", 5, 0),        # stem: Cin 3 (channel padding)
    (2, 64, 14, 14, 128, 1, 1, 0, 1, 1, "int8", "int8", 0, 0),      # 1x1
    (2, 64, 15, 15, 128, 1, 2, 0, 1, 1, "int8", "int8", 7, 0),      # strided 1x1 (downsample)
    (1, 24, 10, 11, 48, 3, 2, (0, 1, 1, 0), 1, 1, "int8", "int8", -8, 0),  # asymmetric pad
    (1, 32, 12, 12, 40, 3, 1, 2, 2, 1, "int8", "int8", 2, 0),       # dilation, ragged Cout
    (1, 32, 8, 8, 64, 3, 1, 1, 1, 1, "uint8", "uint8", 128, 127),   # uint8 both, zw != 0
    (1, 20, 7, 7, 33, 3, 1, 1, 1, 1, "int8", "int8", 1, -2),        # zw != 0, ragged C and O
    (2, 32, 10, 10, 32, 3, 1, 1, 1, 32, "int8", "int8", 3, 0),      # depthwise
    (1, 32, 9, 9, 64, 3, 2, 1, 1, 4, "uint8", "int8", 100, 1),      # grouped, mixed dtypes
    (1, 1, 28, 28, 6, 5, 1, 2, 1, 1, "int8", "int8", -4, 0),        # LeNet conv1 (direct path)
    (3, 256, 7, 7, 512, 3, 1, 1, 1, 1, "int8", "int8", -1, 0),      # K = 2304, image-straddling tiles
    (2, 256, 7, 7, 64, 3, 1, 1, 1, 1, "int8", "int8", 4, 3),        # split-K (small grid) + patch sums
    (1, 160, 6, 6, 48, 3, 1, 1, 1, 1, "uint8", "int8", 130, 0),     # split-K, ragged last split, HW % 4 == 0
]


@pytest.mark.parametrize("case", CONV_CASES, ids=[f"conv{i}" for i in range(len(CONV_CASES))])
def test_conv2d_random(tk, case):
    n, c, h, w, o, k, s, p, d, g, dx, dw_, za, zw = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))  # PYTHONHASHSEED-independent
    x = _rand(rng, (n, c, h, w), dx)
    wt = _rand(rng, (o, c // g, k, k), dw_)
    pad = (p, p, p, p) if isinstance(p, int) else p
    got = tk.conv2d(x, wt, za, zw, strides=(s, s), padding=pad, dilation=(d, d), groups=g)
    exp = ref.qnn_conv2d(x, wt, za, zw, strides=(s, s), padding=pad, dilation=(d, d), groups=g)
    np.testing.assert_array_equal(got, exp)


def test_conv2d_per_channel_kernel_zp(tk):
    rng = np.random.default_rng(7)
    x = _rand(rng, (2, 16, 8, 8), "int8")
    w = _rand(rng, (48, 16, 3, 3), "int8")
    zw = rng.integers(-5, 6, size=48).astype(np.int32)
    got = tk.conv2d(x, w, 3, 0, padding=(1, 1, 1, 1), zw_vec=zw)
    exp = ref.qnn_conv2d(x, w, 3, zw, padding=(1, 1, 1, 1))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("m,k,n,dx,dw_,za,zw", [
    (128, 128, 128, "int8", "int8", -3, 0),
    (1, 400, 120, "int8", "int8", 4, 0),
    (64, 2048, 1000, "int8", "int8", -7, 0),
    (5, 77, 13, "uint8", "uint8", 120, 131),
    (130, 70, 129, "int8", "uint8", 0, 128),
    (16, 1024, 200, "int8", "int8", 5, -3),          # split-K with both zero points
])
def test_dense_random(tk, m, k, n, dx, dw_, za, zw):
    rng = np.random.default_rng(m * 1000 + k)
    x = _rand(rng, (m, k), dx)
    w = _rand(rng, (n, k), dw_)
    np.testing.assert_array_equal(tk.dense(x, w, za, zw), ref.qnn_dense(x, w, za, zw))


@pytest.mark.parametrize("rounding", ["UPWARD", "TONEAREST"])
@pytest.mark.parametrize("out_dtype", ["int8", "uint8", "int32"])
def test_requantize_random(tk, rounding, out_dtype):
    rng = np.random.default_rng(11)
    x = rng.integers(-2**31, 2**31, size=(3, 17, 5, 7), dtype=np.int64).astype(np.int32)
    x[0, 0, 0, :4] = [2**31 - 1, -2**31, 0, -1]
    # per-axis scales incl. a power of two and an equal-to-output one
    s_in = rng.uniform(1e-4, 2.0, size=17).astype(np.float32)
    s_in[0] = 0.125
    s_in[1] = 0.5
    for axis_scale, s_out in ((s_in, np.float32(0.5)), (np.float32(0.0625), np.float32(1.0)),
                              (np.float32(0.3), np.float32(0.7)), (np.float32(3.0), np.float32(1.5))):
        got = tk.requantize(x, axis_scale, np.int32(3), s_out, -2, axis=1, rounding=rounding, out_dtype=out_dtype)
        exp = ref.requantize(x, axis_scale, np.int32(3), s_out, np.int32(-2), axis=1, rounding=rounding,
                             out_dtype=out_dtype)
        np.testing.assert_array_equal(got, exp)


def test_requantize_int8_input_and_vector_zp(tk):
    rng = np.random.default_rng(5)
    x = _rand(rng, (4, 6, 9), "int8")
    zp = rng.integers(-10, 10, size=6).astype(np.int32)
    s = rng.uniform(0.01, 0.1, size=6).astype(np.float32)
    got = tk.requantize(x, s, zp, np.float32(0.05), 7, axis=1)
    exp = ref.requantize(x, s, zp, np.float32(0.05), np.int32(7), axis=1)
    np.testing.assert_array_equal(got, exp)


def test_qnn_add_random(tk):
    rng = np.random.default_rng(3)
    a = _rand(rng, (2, 64, 9, 9), "int8")
    b = _rand(rng, (2, 64, 9, 9), "int8")
    for params in ((0.05, 3, 0.07, -2, 0.09, 1), (0.05, 3, 0.05, 3, 0.05, 3), (0.125, 0, 0.5, 0, 0.25, -5)):
        np.testing.assert_array_equal(tk.qnn_add(a, b, *params), ref.qnn_add(a, b, *params))


ADD_BLOCK_CASES = [
    # shape, dtype, (ls, lz, rs, rz, os, oz), clip, shadow
    ((2, 64, 56, 56), "int8", (0.05, 3, 0.07, -2, 0.09, 1), (1, 127), True),     # HW % 16 == 0, 16-byte path
    ((3, 80, 14, 14), "int8", (0.05, 3, 0.05, 3, 0.05, 3), (3, 127), True),      # HW % 4 == 0, C % 64 != 0
    ((2, 40, 7, 7), "uint8", (0.125, 130, 0.5, 120, 0.25, 128), (128, 255), True),  # HW odd, uint8 xor shadow
    ((2, 24, 9, 9), "int8", (0.02, 0, 0.3, 5, 0.1, -4), None, True),             # no clip: shadow of the add
    ((5, 1000), "int8", (0.05, 3, 0.07, -2, 0.09, 1), (-20, 100), False),        # 2-D, flat view
    ((1, 7, 3, 5), "uint8", (1.0, 0, 1.0, 0, 1.0, 0), None, False),             # both upcast, odd size
]


@pytest.mark.parametrize("case", ADD_BLOCK_CASES, ids=[f"addblock{i}" for i in range(len(ADD_BLOCK_CASES))])
def test_qnn_add_block(tk, case):
    shape, dt, params, clip, want_shadow = case
    rng = np.random.default_rng(len(shape) * 31 + shape[1])
    a = _rand(rng, shape, dt)
    b = _rand(rng, shape, dt)
    outs = tk.qnn_add_block(a, b, *params, clip=clip, want_shadow=want_shadow)
    add = ref.qnn_add(a, b, *params)
    np.testing.assert_array_equal(outs[0], add)
    last = add
    if clip is not None:
        last = ref.clip(add, *clip)
        np.testing.assert_array_equal(outs[1], last)
    if want_shadow:
        np.testing.assert_array_equal(outs[-1], blocked_shadow(last))


def test_elementwise_random(tk):
    rng = np.random.default_rng(9)
    x32 = rng.integers(-2**31, 2**31, size=(3, 5, 7, 3), dtype=np.int64).astype(np.int32)
    bias = rng.integers(-2**31, 2**31, size=(5,), dtype=np.int64).astype(np.int32)
    np.testing.assert_array_equal(tk.bias_add(x32, bias, 1), ref.bias_add(x32, bias, 1))
    x8 = _rand(rng, (2, 3, 33, 5), "int8")
    np.testing.assert_array_equal(tk.unary("tk_clip", x8, None, -3, 100), ref.clip(x8, -3, 100))
    for dst in ("int32", "uint8", "int16"):
        np.testing.assert_array_equal(tk.unary("tk_cast", x32, dst), ref.cast(x32, dst))
    np.testing.assert_array_equal(tk.unary("tk_cast", x8, "int32"), ref.cast(x8, "int32"))


@pytest.mark.parametrize("shape,dt,k,st,pad", [((2, 64, 19, 17), "int8", 3, 2, 1), ((1, 40, 12, 12), "uint8", 3, 2, 1),
                                               ((2, 24, 9, 9), "int8", 2, 2, 0)])
def test_max_pool_from_shadow(tk, shape, dt, k, st, pad):
    rng = np.random.default_rng(shape[1] + k)
    x = _rand(rng, shape, dt)
    rec, sh = tk.max_pool_shadow(x, (k, k), (st, st), (pad,) * 4)
    exp = ref.max_pool2d(x, (k, k), (st, st), (pad,) * 4)
    np.testing.assert_array_equal(rec, exp)
    np.testing.assert_array_equal(sh, blocked_shadow(exp))


def test_pools(tk):
    rng = np.random.default_rng(4)
    x8 = _rand(rng, (2, 5, 13, 11), "int8")
    np.testing.assert_array_equal(tk.pool("tk_max_pool2d", x8, (3, 3), (2, 2), (1, 1, 1, 1)),
                                  ref.max_pool2d(x8, (3, 3), (2, 2), (1, 1, 1, 1)))
    np.testing.assert_array_equal(tk.pool("tk_max_pool2d", x8, (2, 2), (2, 2), (0, 0, 0, 0)),
                                  ref.max_pool2d(x8, (2, 2), (2, 2), (0, 0, 0, 0)))
    x32 = rng.integers(-10**6, 10**6, size=(2, 5, 13, 11)).astype(np.int32)
    for cip in (False, True):
        np.testing.assert_array_equal(tk.pool("tk_avg_pool2d", x32, (3, 3), (2, 2), (1, 1, 1, 1), count_include_pad=cip),
                                      ref.avg_pool2d(x32, (3, 3), (2, 2), (1, 1, 1, 1), count_include_pad=cip))
    x32 = rng.integers(-10**6, 10**6, size=(3, 7, 7, 7)).astype(np.int32)
    np.testing.assert_array_equal(tk.global_avg_pool(x32), ref.global_avg_pool2d(x32))


BLOCK_CASES = [
    # N, C, H, W, O, K, stride, pad, groups, dx, za, out_dtype, clip
    (2, 32, 9, 9, 64, 3, 1, 1, 1, "int8", -3, "int8", (2, 127)),
    (1, 3, 15, 15, 64, 7, 2, 3, 1, "int8", 4, "int8", (-5, 100)),
    (2, 64, 7, 7, 200, 1, 1, 0, 1, "uint8", 130, "uint8", None),
    (1, 24, 10, 10, 24, 3, 2, 1, 24, "int8", 1, "int8", (0, 96)),     # depthwise (direct kernel)
    (1, 1, 12, 12, 6, 5, 1, 2, 1, "int8", 0, "int8", (-1, 127)),      # tiny Cin (direct kernel)
    (2, 128, 7, 7, 256, 3, 1, 1, 1, "int8", -2, "int8", (0, 127)),    # split-K block, scalar-store epilogue
    (4, 256, 14, 14, 96, 1, 2, 0, 1, "int8", 5, "uint8", None),       # split-K strided 1x1, 7x7 out
    (40, 32, 4, 4, 64, 3, 2, 1, 1, "int8", 1, "int8", (0, 127)),      # 2x2 planes: 32 images per tile
    (7, 16, 5, 5, 36, 3, 1, 1, 1, "uint8", 128, "uint8", None),       # 5x5 planes, last tile partial
    (2, 512, 7, 7, 64, 3, 1, 1, 1, "int8", -3, "int8", (0, 127)),     # 128-byte K stages + split-K
    (2, 256, 14, 14, 128, 3, 1, 1, 1, "int8", 2, "int8", None),       # 128-byte K stages, 128-column tiles
    (2, 128, 9, 9, 64, 3, 1, 1, 1, "uint8", 130, "uint8", (128, 255)),  # 128-byte K stages, uint8
    (2, 128, 12, 12, 128, 3, 1, 1, 1, "int8", 3, "int8", (0, 127)),   # 128 channels, K >= 512: 128-row tiles
    (3, 512, 6, 6, 128, 1, 1, 0, 1, "uint8", 129, "uint8", None),     # 128-row tiles, 1x1, uint8
    (150, 256, 1, 1, 200, 1, 1, 0, 1, "int8", 2, "int8", (0, 127)),   # 1x1 planes (a dense layer): 128 images per tile
    (9, 64, 3, 3, 64, 3, 1, 1, 1, "int8", -1, "int8", None),          # 3x3 planes: up to 3 row changes per group
    (2, 64, 56, 56, 64, 3, 1, 1, 64, "int8", 3, "int8", (0, 127)),    # depthwise band kernel, 4-pixel vectors, last band partial
    (1, 16, 112, 112, 16, 3, 2, 1, 16, "uint8", 130, "uint8", (128, 255)),  # depthwise stride 2, uint8
    (3, 32, 14, 14, 32, 3, 1, 1, 32, "int8", -4, "int8", None),       # depthwise, whole plane per group, scalar pixels
    (2, 64, 7, 7, 64, 1, 1, 0, 1, "int8", 1, "int8", (100, 20)),      # a_min > a_max: clip gives a_min (flat epilogue)
    (2, 64, 16, 16, 64, 1, 1, 0, 1, "uint8", 129, "uint8", (200, 150)),  # a_min > a_max, 4-column epilogue
]


# stride-1 3x3 blocks of ResNet stage shapes: whole-image tiles of the image-tile kernel on planes of
# up to 256 pixels (several images per workgroup, the last one partial), the im2col kernel's tiles
# on the 28x28 / 56x56 / 20x20 planes
HALO_CASES = [
    # N, C, H, O, dx, za, out_dtype, clip
    (3, 64, 28, 128, "int8", -3, "int8", (0, 127)),
    (2, 64, 56, 64, "int8", 4, "int8", (2, 127)),
    (5, 256, 14, 256, "int8", 1, "int8", (0, 127)),
    (3, 512, 7, 512, "int8", -2, "int8", (0, 127)),
    (40, 64, 6, 64, "uint8", 131, "uint8", (128, 255)),
    (1, 128, 14, 192, "uint8", 125, "uint8", None),
    (2, 192, 20, 64, "int8", 0, "int8", (-7, 99)),
]


@pytest.mark.parametrize("case", HALO_CASES, ids=[f"halo{i}" for i in range(len(HALO_CASES))])
def test_conv3x3_halo_block(tk, case):
    n, c, h, o, dx, za, odt, clip = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    x = _rand(rng, (n, c, h, h), dx)
    wt = _rand(rng, (o, c, 3, 3), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_in = rng.uniform(1e-5, 1e-3, size=o).astype(np.float32)
    s_out = np.float32(0.01)
    pad = (1, 1, 1, 1)
    outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, clip=clip, padding=pad, out_dtype=odt,
                           want_shadow=True)
    conv = ref.qnn_conv2d(x, wt, za, 0, padding=pad)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=odt)
    exp = [conv, badd, rq] + ([ref.clip(rq, *clip)] if clip is not None else [])
    for got, e in zip(outs, exp):
        np.testing.assert_array_equal(got, e)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


# 1x1 / 3x3 blocks of every ResNet stage shape: strided 1x1 (downsample) and strided 3x3,
# residual joins, expand layers (1x1 to 4x the channels), 32-channel output multiples (96), uint8
PATCH_CASES = [
    # N, C, H, O, K, stride, dx, za, residual add params or None, clip
    (3, 256, 28, 512, 1, 2, "int8", -2, None, None),
    (2, 512, 14, 1024, 1, 2, "int8", 3, None, None),
    (3, 128, 28, 128, 3, 2, "int8", 1, None, (0, 127)),
    (2, 512, 14, 512, 3, 2, "int8", -1, None, (0, 127)),
    (3, 64, 56, 256, 1, 1, "int8", 2, (0.05, -3, 0.06, 4, 0.08, -1), (-1, 127)),
    (2, 128, 28, 512, 1, 1, "int8", -4, (0.05, 3, 0.07, -2, 0.09, 1), (1, 127)),
    (5, 256, 14, 1024, 1, 1, "int8", 1, (0.04, 0, 0.04, 0, 0.04, 0), (0, 127)),
    (3, 512, 7, 2048, 1, 1, "uint8", 130, (0.1, 130, 0.2, 120, 0.15, 128), (128, 255)),
    (2, 1024, 14, 256, 1, 1, "int8", 2, None, (0, 127)),
    (3, 2048, 7, 512, 1, 1, "int8", -3, None, (0, 127)),
    (2, 64, 56, 64, 1, 1, "int8", 5, None, (0, 127)),
    (4, 192, 10, 96, 3, 1, "int8", 0, (0.05, -3, 0.06, 4, 0.08, -1), None),
]


@pytest.mark.parametrize("case", PATCH_CASES, ids=[f"patch{i}" for i in range(len(PATCH_CASES))])
def test_conv_patch_block(tk, case):
    n, c, h, o, k, st, dt, za, ap, clip = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    x = _rand(rng, (n, c, h, h), dt)
    wt = _rand(rng, (o, c, k, k), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_in = rng.uniform(1e-5, 1e-3, size=o).astype(np.float32)
    s_out = np.float32(0.01)
    p = k // 2
    pad = (p, p, p, p)
    oh = (h + 2 * p - k) // st + 1
    residual = _rand(rng, (n, o, oh, oh), dt) if ap is not None else None
    outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, clip=clip, strides=(st, st), padding=pad,
                           out_dtype=dt, want_shadow=True, residual=residual, add_params=ap)
    conv = ref.qnn_conv2d(x, wt, za, 0, strides=(st, st), padding=pad)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=dt)
    exp = [conv, badd, rq]
    if ap is not None:
        exp.append(ref.qnn_add(rq, residual, *ap))
    if clip is not None:
        exp.append(ref.clip(exp[-1], *clip))
    for got, e in zip(outs, exp):
        np.testing.assert_array_equal(got, e)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


# image-tile kernel (tk_conv_img.hip): 1x1 (128-channel stages) and 3x3 (32-channel stages, chunked
# weights) blocks on planes of up to 256 pixels, R = 64 / 32 output channels x whole images per
# workgroup; several images per workgroup with the last one ragged, planes whose pixel count is
# not a multiple of 4 (groups crossing channel rows), strided 3x3 (halo of a strided patch) and
# strided 1x1 (strided patch loader), residual joins on either side, uint8, no clip
IMG_CASES = [
    # N, C, H, O, K, stride, dtype, za, residual add params or None, clip, block_is_rhs
    (5, 256, 14, 256, 3, 1, "int8", -3, None, (0, 127), False),
    (3, 512, 7, 512, 3, 1, "int8", 2, None, (0, 127), False),
    (7, 64, 7, 96, 3, 1, "uint8", 130, None, (128, 255), False),
    (3, 96, 9, 64, 3, 1, "int8", 1, (0.05, -3, 0.06, 4, 0.08, -1), (-1, 127), False),
    (4, 128, 16, 128, 3, 1, "int8", 0, None, None, False),
    (3, 256, 14, 128, 3, 2, "int8", 4, None, (0, 127), False),
    (2, 128, 28, 64, 3, 2, "uint8", 129, None, None, False),
    (2, 128, 12, 64, 3, 1, "int8", 2, (0.05, 3, 0.07, -2, 0.09, 1), (1, 127), True),
    (6, 1024, 14, 256, 1, 1, "int8", 2, None, (0, 127), False),
    (5, 256, 14, 1024, 1, 1, "int8", -1, (0.04, 0, 0.04, 0, 0.04, 0), (0, 127), False),
    (3, 512, 7, 2048, 1, 1, "uint8", 130, (0.1, 130, 0.2, 120, 0.15, 128), (128, 255), True),
    (4, 512, 28, 1024, 1, 2, "int8", 3, None, None, False),
    (3, 2048, 7, 512, 1, 1, "int8", -2, None, (0, 127), False),
    (9, 128, 5, 64, 1, 1, "int8", 5, (0.05, -3, 0.06, 4, 0.08, -1), None, False),
]


@pytest.mark.parametrize("case", IMG_CASES, ids=[f"img{i}" for i in range(len(IMG_CASES))])
def test_conv_img_block(tk, case):
    """Every record (and the shadow of the last one) of a block on the image-tile kernel against
    the unfused oracle ops."""
    n, c, h, o, k, st, dt, za, ap, clip, rhs = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    x = _rand(rng, (n, c, h, h), dt)
    wt = _rand(rng, (o, c, k, k), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_in = rng.uniform(1e-5, 1e-3, size=o).astype(np.float32)
    s_out = np.float32(0.01)
    p = k // 2
    pad = (p, p, p, p)
    oh = (h + 2 * p - k) // st + 1
    kw = dict(clip=clip, strides=(st, st), padding=pad, out_dtype=dt, want_shadow=True)
    residual = None
    if ap is not None:
        residual = _rand(rng, (n, o, oh, oh), dt)
        kw.update(residual=residual, add_params=ap, block_is_rhs=rhs)
    outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, **kw)
    conv = ref.qnn_conv2d(x, wt, za, 0, strides=(st, st), padding=pad)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=dt)
    exp = [conv, badd, rq]
    if ap is not None:
        exp.append(ref.qnn_add(residual, rq, *ap) if rhs else ref.qnn_add(rq, residual, *ap))
    if clip is not None:
        exp.append(ref.clip(exp[-1], *clip))
    for got, e in zip(outs, exp):
        np.testing.assert_array_equal(got, e)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


# every kernel a block can run on (tk_conv2d_block_algos: im2col tiles and each image-tile plan --
# R = 32 / 64 rows, 32 / 64 / 128-channel stages, 1..28 images per workgroup, one or two workgroups
# per CU), incl. the 28x28 planes that only R = 32 x 7 column tiles per wave cover
ALGO_CASES = [
    # N, C, H, O, K, stride, dtype, za, residual add params or None, clip
    (3, 128, 28, 128, 3, 1, "int8", -2, None, (0, 127)),
    (2, 128, 28, 512, 1, 1, "int8", 3, (0.05, 3, 0.07, -2, 0.09, 1), (1, 127)),
    (3, 256, 14, 1024, 1, 1, "uint8", 131, (0.1, 130, 0.2, 120, 0.15, 128), (128, 255)),
    (4, 256, 14, 256, 3, 1, "int8", 1, None, (0, 127)),
    (5, 512, 7, 512, 3, 1, "int8", -1, None, (0, 127)),
    (3, 256, 56, 512, 1, 2, "int8", 2, None, None),
    (2, 64, 28, 96, 1, 1, "int8", 0, None, (0, 127)),
    # 56x56 (the persistent kernel's home): K = 64 (one stage; 800 tiles, so workgroups of both
    # ring sizes walk several), 3x3 over 64 channels (9 stages; 296 tiles)
    (8, 64, 56, 256, 1, 1, "int8", 1, (0.05, 3, 0.07, -2, 0.09, 1), (0, 127)),
    (12, 64, 56, 64, 3, 1, "int8", 0, None, (0, 127)),
    # requantize scales near 1 (shift > -2: the general requantize form, not the mul_hi one)
    (2, 128, 28, 128, 1, 1, "int8", 2, None, (0, 127), (0.005, 0.03)),
    # 3x3 with 64-channel K stages: an odd number of stages (3, stride 2) through the two-slot ring,
    # and 5 stages of a uint8 block with a residual join on a 7x7 plane
    (3, 192, 14, 64, 3, 2, "int8", 0, None, (0, 127)),
    (2, 320, 7, 64, 3, 1, "uint8", 129, (0.1, 130, 0.2, 120, 0.15, 128), (128, 255)),
    # round 4: split-K image plans over a stage count no split divides (5 stages of 32 channels),
    # and a stride-2 3x3 on an odd input width (no column-parity patch), uint8 with a residual join
    (4, 160, 7, 64, 3, 1, "int8", -3, None, (0, 127)),
    (2, 64, 13, 64, 3, 2, "uint8", 131, (0.1, 130, 0.2, 120, 0.15, 128), (128, 255)),
    # round 6, the weight-stationary 1x1 kernel (algo 6): a partial last 32-row chunk under a uint8
    # residual join (MobileNetV2's 24 -> 144), and 40 channels (a partial 16-channel shadow group)
    # on a plane that several tiles share
    (3, 24, 28, 144, 1, 1, "uint8", 131, (0.1, 130, 0.2, 120, 0.15, 128), (128, 255)),
    (2, 32, 20, 40, 1, 1, "int8", 2, (0.05, 3, 0.07, -2, 0.09, 1), None),
    # dense heads as 1x1 blocks over [B, K, 1, 1] (the dense tile kernel, algo 5): ResNet-50's
    # 2048 -> 1000 over 8 K slices, and a ragged 40-sample uint8 batch
    (64, 2048, 1, 1000, 1, 1, "int8", -3, None, (0, 127)),
    (40, 512, 1, 96, 1, 1, "uint8", 131, None, None),
]


@pytest.mark.parametrize("case", ALGO_CASES, ids=[f"algo{i}" for i in range(len(ALGO_CASES))])
def test_conv_block_every_algo(tk, case):
    """Each algo tk_conv2d_block_algos lists gives the oracle's records bit for bit."""
    n, c, h, o, k, st, dt, za, ap, clip = case[:10]
    s_lo, s_hi = case[10] if len(case) > 10 else (1e-5, 1e-3)
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    x = _rand(rng, (n, c, h, h), dt)
    wt = _rand(rng, (o, c, k, k), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_in = rng.uniform(s_lo, s_hi, size=o).astype(np.float32)
    s_out = np.float32(0.01)
    p = k // 2
    pad = (p, p, p, p)
    oh = (h + 2 * p - k) // st + 1
    kw = dict(clip=clip, strides=(st, st), padding=pad, out_dtype=dt, want_shadow=True)
    residual = None
    if ap is not None:
        residual = _rand(rng, (n, o, oh, oh), dt)
        kw.update(residual=residual, add_params=ap)
    algos = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, algos_only=True, **kw)
    # im2col tiles always; dense heads list the dense tile kernel (5) first
    assert 1 in algos and algos[0] in (1, 5) and len(algos) >= 2, algos
    conv = ref.qnn_conv2d(x, wt, za, 0, strides=(st, st), padding=pad)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=dt)
    exp = [conv, badd, rq]
    if ap is not None:
        exp.append(ref.qnn_add(rq, residual, *ap))
    if clip is not None:
        exp.append(ref.clip(exp[-1], *clip))
    exp.append(blocked_shadow(exp[-1]))
    bad = []
    for algo in [0] + algos:
        outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, algo=algo, **kw)
        for i, (got, e) in enumerate(zip(outs, exp)):
            if not np.array_equal(got, e):
                where = np.argwhere(got != e)
                bad.append(f"algo {algo} output {i}: {len(where)} of {e.size} differ, first at {where[0].tolist()}, "
                           f"index ranges {where.min(0).tolist()}..{where.max(0).tolist()}")
    assert not bad, "\n".join(bad)


def test_conv_block_bad_algo(tk):
    """An algo the block does not have fails loudly (no silent fallback)."""
    rng = np.random.default_rng(5)
    x = _rand(rng, (2, 64, 14, 14), "int8")
    wt = _rand(rng, (64, 64, 1, 1), "int8")
    bias = np.zeros(64, np.int32)
    s_in = np.full(64, 1e-4, np.float32)
    n_algos = len(tk.conv2d_block(x, wt, bias, 1, 0, s_in, np.float32(0.01), 3, algos_only=True))
    with pytest.raises(Exception, match="does not apply"):
        tk.conv2d_block(x, wt, bias, 1, 0, s_in, np.float32(0.01), 3, algo=16 + n_algos)


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("rounding", ["UPWARD", "TONEAREST"])
def test_conv_img_shift_regimes(tk, rounding, k):
    """The image-tile kernel's general requantize path (per-channel right shifts 0..8 and left
    shifts) and TONEAREST, against the oracle."""
    rng = np.random.default_rng(79 + k)
    n, c, h, o = 3, 128, 14, 64
    x = _rand(rng, (n, c, h, h), "int8")
    wt = _rand(rng, (o, c, k, k), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_out = np.float32(0.5)
    s_in = (np.geomspace(2.0 ** -8, 3.5, o) * s_out).astype(np.float32)
    pad = (k // 2,) * 4
    outs = tk.conv2d_block(x, wt, bias, 3, 0, s_in, s_out, -4, clip=(-128, 127), padding=pad, rounding=rounding,
                           want_shadow=True)
    conv = ref.qnn_conv2d(x, wt, 3, 0, padding=pad)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(-4), axis=1, out_dtype="int8", rounding=rounding)
    for got, e in zip(outs, [conv, badd, rq, rq]):
        np.testing.assert_array_equal(got, e)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(rq))


@pytest.mark.parametrize("rounding", ["UPWARD", "TONEAREST"])
def test_conv3x3_halo_shift_regimes(tk, rounding):
    """The halo kernel's general requantize path (right shifts 0..8, left shifts) and the
    TONEAREST rounding, against the oracle."""
    rng = np.random.default_rng(78)
    n, c, h, o = 2, 64, 14, 64
    x = _rand(rng, (n, c, h, h), "int8")
    wt = _rand(rng, (o, c, 3, 3), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_out = np.float32(0.5)
    s_in = (np.geomspace(2.0 ** -8, 3.5, o) * s_out).astype(np.float32)
    outs = tk.conv2d_block(x, wt, bias, 3, 0, s_in, s_out, -4, clip=(-128, 127), padding=(1, 1, 1, 1),
                           rounding=rounding, want_shadow=True)
    conv = ref.qnn_conv2d(x, wt, 3, 0, padding=(1, 1, 1, 1))
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(-4), axis=1, out_dtype="int8", rounding=rounding)
    for got, e in zip(outs, [conv, badd, rq, rq]):
        np.testing.assert_array_equal(got, e)


def test_conv_block_requantize_shift_regimes(tk):
    """Per-channel multipliers spanning right shifts 0..8 and left shifts 1..2, so the block
    epilogue's mul_hi fast path (right shift >= 2) and the general int64 path both run,
    against the oracle on the same inputs."""
    rng = np.random.default_rng(77)
    n, c, h, w, o = 2, 64, 8, 8, 64
    x = _rand(rng, (n, c, h, w), "int8")
    wt = _rand(rng, (o, c, 1, 1), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_out = np.float32(0.5)
    mult = np.geomspace(2.0 ** -8, 3.5, o)  # M = s_in / s_out
    s_in = (mult * s_out).astype(np.float32)
    outs = tk.conv2d_block(x, wt, bias, 3, 0, s_in, s_out, -4, clip=(-128, 127), want_shadow=True)
    conv = ref.qnn_conv2d(x, wt, 3, 0)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(-4), axis=1, out_dtype="int8")
    for got, e in zip(outs, [conv, badd, rq, rq]):
        np.testing.assert_array_equal(got, e)


RESIDUAL_CASES = [
    # N, C, H, W, O, K, stride, pad, dtype, add params (lhs s/zp, rhs s/zp, out s/zp), clip, block_is_rhs
    (2, 32, 8, 8, 128, 1, 1, 0, "int8", (0.05, 3, 0.07, -2, 0.09, 1), (1, 127), False),
    (2, 32, 8, 8, 128, 1, 1, 0, "int8", (0.05, 3, 0.07, -2, 0.09, 1), (1, 127), True),
    (2, 64, 7, 7, 96, 3, 1, 1, "int8", (0.04, 0, 0.04, 0, 0.04, 0), None, False),     # both upcast, scalar stores
    (1, 48, 12, 12, 64, 3, 1, 1, "uint8", (0.1, 130, 0.2, 120, 0.15, 128), (128, 255), True),
    (2, 256, 7, 7, 128, 3, 1, 1, "int8", (0.05, -3, 0.06, 4, 0.08, -1), (-1, 127), False),  # split-K
    (2, 512, 10, 10, 128, 1, 1, 0, "int8", (0.05, -3, 0.06, 4, 0.08, -1), (0, 127), True),  # 128-row tiles
    (70, 64, 1, 1, 96, 1, 1, 0, "uint8", (0.1, 130, 0.2, 120, 0.15, 128), (128, 255), True),  # 1x1 planes
]


@pytest.mark.parametrize("case", RESIDUAL_CASES, ids=[f"resid{i}" for i in range(len(RESIDUAL_CASES))])
def test_conv_block_residual_join(tk, case):
    """conv -> bias_add -> requantize -> qnn.add(., residual) [-> clip] in one block kernel, every
    record plus the shadow of the last one against the unfused oracle ops."""
    n, c, h, w, o, k, s, p, dt, ap, clip, rhs = case
    rng = np.random.default_rng(1000 + o + k)
    x = _rand(rng, (n, c, h, w), dt)
    wt = _rand(rng, (o, c, k, k), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_in = rng.uniform(1e-5, 1e-3, size=o).astype(np.float32)
    s_out = np.float32(0.01)
    za = 130 if dt == "uint8" else 2
    oh = (h + 2 * p - k) // s + 1
    residual = _rand(rng, (n, o, oh, oh), dt)
    outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, clip=clip, strides=(s, s), padding=(p, p, p, p),
                           out_dtype=dt, want_shadow=True, residual=residual, add_params=ap, block_is_rhs=rhs)
    conv = ref.qnn_conv2d(x, wt, za, 0, strides=(s, s), padding=(p, p, p, p))
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=dt)
    add = ref.qnn_add(residual, rq, *ap) if rhs else ref.qnn_add(rq, residual, *ap)
    exp = [conv, badd, rq, add]
    if clip is not None:
        exp.append(ref.clip(add, *clip))
    for got, e in zip(outs, exp):
        np.testing.assert_array_equal(got, e)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


# 256-column image tiles (planes of 65..256 pixels, K <= 256, grids of >= 256 tiles): one image per
# tile on 14x14 / 12x12 planes, two on 10x10 and three on 9x9 (last tile ragged), strided 1x1
# (downsample 28 -> 14), residual joins, uint8, the general im2col walk (Cin not a multiple of 64)
BN256_CASES = [
    # N, C, H, O, K, stride, pad, dtype, residual add params or None, clip
    (16, 64, 14, 1024, 1, 1, 0, "int8", (0.05, 3, 0.07, -2, 0.09, 1), (0, 127)),
    (32, 256, 12, 512, 1, 1, 0, "int8", None, (0, 127)),
    (33, 64, 10, 1024, 1, 1, 0, "uint8", (0.1, 130, 0.2, 120, 0.15, 128), (128, 255)),
    (16, 128, 28, 1024, 1, 2, 0, "int8", None, None),
    (16, 512, 28, 1024, 1, 2, 0, "int8", None, (0, 127)),               # K = 512 (TK_BN256_KMAX A/Bs)
    (48, 32, 9, 1024, 3, 1, 1, "int8", None, (-3, 120)),
    (64, 256, 14, 256, 1, 1, 0, "int8", (0.04, 0, 0.04, 0, 0.04, 0), None),
    # planes > 256 pixels, >= 256 channels (256-column row tiles with TK_BN256_ROWS=1 in the
    # ablation build, 128-column tiles in the product): tiles cross images, the last one ragged;
    # residual join, uint8, strided downsample
    (2, 64, 96, 256, 1, 1, 0, "int8", (0.05, 3, 0.07, -2, 0.09, 1), (0, 127)),
    (12, 128, 28, 512, 1, 1, 0, "uint8", (0.1, 130, 0.2, 120, 0.15, 128), (128, 255)),
    (12, 256, 56, 512, 1, 2, 0, "int8", None, None),
]


@pytest.mark.parametrize("case", BN256_CASES, ids=[f"bn256_{i}" for i in range(len(BN256_CASES))])
def test_conv_block_bn256(tk, case):
    """Every record (and the shadow of the last one) of a block on 256-column image tiles
    against the unfused oracle ops."""
    n, c, h, o, k, s, p, dt, ap, clip = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    x = _rand(rng, (n, c, h, h), dt)
    wt = _rand(rng, (o, c, k, k), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_in = rng.uniform(1e-5, 1e-3, size=o).astype(np.float32)
    s_out = np.float32(0.01)
    za = 130 if dt == "uint8" else 2
    oh = (h + 2 * p - k) // s + 1
    kw = dict(clip=clip, strides=(s, s), padding=(p, p, p, p), out_dtype=dt, want_shadow=True)
    residual = None
    if ap is not None:
        residual = _rand(rng, (n, o, oh, oh), dt)
        kw.update(residual=residual, add_params=ap, block_is_rhs=False)
    outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, **kw)
    conv = ref.qnn_conv2d(x, wt, za, 0, strides=(s, s), padding=(p, p, p, p))
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=dt)
    exp = [conv, badd, rq]
    if ap is not None:
        exp.append(ref.qnn_add(rq, residual, *ap))
    if clip is not None:
        exp.append(ref.clip(exp[-1], *clip))
    for got, e in zip(outs, exp):
        np.testing.assert_array_equal(got, e)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


@pytest.mark.parametrize("dt", ["int8", "uint8"])
def test_conv_block_mt2_256(tk, dt):
    """ResNet-50's 14x14 3x3 256->256 layer at batch 64 on 128-row tiles (K = 2304, 196 tiles): every
    record and the shadow against the oracle (the C restatement of the conv, for its size)."""
    from oracle import graph_ref
    rng = np.random.default_rng(zlib.crc32(f"mt2_256 {dt}".encode()))
    x = _rand(rng, (64, 256, 14, 14), dt)
    wt = _rand(rng, (256, 256, 3, 3), "int8")
    bias = rng.integers(-2**14, 2**14, size=256).astype(np.int32)
    s_in = rng.uniform(1e-5, 1e-4, size=256).astype(np.float32)
    s_out = np.float32(0.02)
    za = 131 if dt == "uint8" else -3
    clip = (128, 255) if dt == "uint8" else (0, 127)
    outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, clip=clip, padding=(1, 1, 1, 1), out_dtype=dt,
                           want_shadow=True)
    conv = graph_ref._conv_c(x, wt, za, 0, {"strides": (1, 1), "dilation": (1, 1), "padding": (1, 1, 1, 1),
                                            "groups": 1}, 16)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=dt)
    exp = [conv, badd, rq, ref.clip(rq, *clip)]
    for got, e in zip(outs, exp):
        np.testing.assert_array_equal(got, e)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


@pytest.mark.parametrize("case", BLOCK_CASES, ids=[f"block{i}" for i in range(len(BLOCK_CASES))])
def test_conv_block_matches_unfused_ops(tk, case):
    n, c, h, w, o, k, s, p, g, dx, za, odt, clip = case
    rng = np.random.default_rng(17 + n * c)
    x = _rand(rng, (n, c, h, w), dx)
    wt = _rand(rng, (o, c // g, k, k), "int8")
    bias = rng.integers(-2**14, 2**14, size=o).astype(np.int32)
    s_in = rng.uniform(1e-5, 1e-3, size=o).astype(np.float32)
    s_out = np.float32(0.01)
    pad = (p, p, p, p)
    outs = tk.conv2d_block(x, wt, bias, za, 0, s_in, s_out, 3, clip=clip, strides=(s, s), padding=pad, groups=g,
                           out_dtype=odt, want_shadow=True)
    conv = ref.qnn_conv2d(x, wt, za, 0, strides=(s, s), padding=pad, groups=g)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, out_dtype=odt)
    exp = [conv, badd, rq]
    if clip is not None:
        exp.append(ref.clip(rq, *clip))
    for got, e in zip(outs, exp):
        np.testing.assert_array_equal(got, e)
    # the shadow of the last output (what the next MFMA conv reads)
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


# depthwise 3x3 blocks on the tile kernel (tk_dw.hip): every MobileNetV2 depthwise shape class --
# 112 / 56 planes in row bands (last band partial), whole 28 / 14 planes, 7x7 planes four channel
# groups per tile (flat 4-element groups crossing rows and channels), stride 1 and 2, valid padding,
# odd planes -- with uint8 data / weights, scalar and per-channel kernel zero points, per-tensor
# and per-axis requantize, both roundings and the general (right shift < 2) requantize form
DW_CASES = [
    # N, C, H, W, stride, pad, dx, dw, za, zw ("vec": per channel), s_in ("axis" | scalar), rounding, out, clip
    (2, 32, 112, 112, 1, 1, "int8", "int8", 3, 0, "axis", "UPWARD", "int8", (0, 127)),
    (1, 96, 112, 112, 2, 1, "int8", "int8", -5, 0, "axis", "UPWARD", "int8", (0, 127)),
    (2, 144, 56, 56, 1, 1, "int8", "int8", 0, 0, "axis", "UPWARD", "int8", (0, 127)),
    (2, 144, 56, 56, 2, 1, "int8", "int8", 7, 0, "axis", "TONEAREST", "int8", (0, 127)),
    (2, 192, 28, 28, 1, 1, "int8", "int8", -1, 0, "axis", "UPWARD", "int8", (0, 127)),
    (3, 192, 28, 28, 2, 1, "int8", "int8", 2, 0, "axis", "UPWARD", "int8", (0, 127)),
    (2, 384, 14, 14, 1, 1, "int8", "int8", -8, 0, "axis", "UPWARD", "int8", (0, 127)),
    (2, 576, 14, 14, 2, 1, "int8", "int8", 4, 0, "axis", "UPWARD", "int8", (0, 127)),
    (2, 960, 7, 7, 1, 1, "int8", "int8", 1, 0, "axis", "UPWARD", "int8", (0, 127)),
    (1, 48, 7, 7, 1, 1, "int8", "int8", 1, 0, "axis", "UPWARD", "int8", None),
    (2, 32, 28, 28, 1, 1, "uint8", "uint8", 130, 3, "axis", "UPWARD", "uint8", (128, 255)),
    (2, 64, 14, 14, 2, 1, "int8", "int8", -2, "vec", "axis", "UPWARD", "int8", (0, 127)),
    (2, 32, 30, 30, 1, 0, "int8", "uint8", 5, 120, "axis", "UPWARD", "int8", (-3, 90)),
    (2, 16, 20, 20, 1, 1, "int8", "int8", 0, 0, 0.5, "TONEAREST", "int8", None),
    (2, 16, 9, 9, 2, 1, "uint8", "int8", 125, 0, 0.0007, "UPWARD", "uint8", (130, 250)),
    # full-batch shapes whose plans differ from the small-batch ones: row bands of 14-wide planes
    # (flat groups, 6-row bands and a 2-row last band) and 28-wide bands with many tiles
    (64, 192, 28, 28, 2, 1, "int8", "int8", 2, 0, "axis", "UPWARD", "int8", (0, 127)),
    (64, 192, 28, 28, 1, 1, "int8", "int8", -3, 0, "axis", "UPWARD", "int8", (0, 127)),
    # round 6, the flat staging of narrow whole planes: four 16-channel groups of 7x7 planes per
    # tile at the full batch, and a stride-2 unpadded 14x14 plane whose staged rows stop short of the
    # last input row (the row-load staging keeps it)
    (64, 960, 7, 7, 1, 1, "int8", "int8", -4, 0, "axis", "UPWARD", "int8", (0, 127)),
    (2, 16, 14, 14, 2, 0, "uint8", "int8", 120, 0, "axis", "UPWARD", "uint8", None),
]


@pytest.mark.parametrize("case", DW_CASES, ids=[f"dw{i}" for i in range(len(DW_CASES))])
def test_depthwise_block(tk, case):
    n, c, h, w, st, p, dx, dw_, za, zw, sk, rounding, odt, clip = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    x = _rand(rng, (n, c, h, w), dx)
    wt = _rand(rng, (c, 1, 3, 3), dw_)
    bias = rng.integers(-2**14, 2**14, size=c).astype(np.int32)
    s_in = rng.uniform(1e-4, 3e-3, size=c).astype(np.float32) if sk == "axis" else np.float32(sk)
    s_out = np.float32(0.01)
    zv = rng.integers(-6, 7, size=c).astype(np.int32) if zw == "vec" else None
    zs = 0 if zw == "vec" else zw
    pad = (p, p, p, p)
    outs = tk.conv2d_block(x, wt, bias, za, zs, s_in, s_out, 3, clip=clip, strides=(st, st), padding=pad, groups=c,
                           out_dtype=odt, want_shadow=True, rounding=rounding, zw_vec=zv)
    conv = ref.qnn_conv2d(x, wt, za, zv if zv is not None else zs, strides=(st, st), padding=pad, groups=c)
    badd = ref.bias_add(conv, bias, 1)
    rq = ref.requantize(badd, s_in, np.int32(0), s_out, np.int32(3), axis=1, rounding=rounding, out_dtype=odt)
    exp = [conv, badd, rq] + ([ref.clip(rq, *clip)] if clip is not None else [])
    for i, (got, e) in enumerate(zip(outs, exp)):
        if not np.array_equal(got, e):
            bad = np.argwhere(got != e)[0]
            raise AssertionError(f"record {i}: {int((got != e).sum())} mismatches, first at {tuple(bad)}: "
                                 f"{got[tuple(bad)]} vs {e[tuple(bad)]}")
    np.testing.assert_array_equal(outs[-1], blocked_shadow(exp[-1]))


@pytest.mark.parametrize("dt,value", [("int8", -5), ("uint8", 200), ("int32", -70000), ("float32", 1.5)])
def test_pad(tk, dt, value):
    """tk_pad (nn.pad, constant mode) against the oracle's np.pad restatement."""
    from tachikoma_amd import _lib
    rng = np.random.default_rng(31)
    x = _rand(rng, (2, 3, 5, 7), dt) if dt != "float32" else rng.standard_normal((2, 3, 5, 7)).astype(np.float32)
    pw = ((0, 1), (1, 2), (3, 0), (2, 2))
    exp = ref.pad(x, pw, np.asarray(value).astype(dt))
    out = tk.empty(exp.shape, dt)
    a = _lib.tk_pad_attrs()
    for d, (b, e) in enumerate(pw):
        a.before[d], a.after[d] = b, e
    if dt == "float32":
        a.value_f = value
    else:
        a.value_i = int(np.asarray(value).astype(dt).astype(np.int64))
    xd = tk.dev(x)
    rc = _lib.load().tk_pad(tk.ref(xd).ptr, tk.ref(out).ptr, a, tk.stream())
    tk._sync_check(rc, "tk_pad")
    np.testing.assert_array_equal(out.cpu().numpy(), exp)

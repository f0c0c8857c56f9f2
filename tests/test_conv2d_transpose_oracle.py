"""An independent restatement of qnn.conv2d_transpose checks oracle/qnn_ref.qnn_conv2d_transpose.

The oracle's gather form and the device kernel share one reading of legalizations.py; this test
restates the op the way topi computes it instead (python/tvm/topi/nn/conv2d_transpose.py,
conv2d_transpose_nchw_preprocess): shift both operands by their zero points (the x86 int16
legalization, python/tvm/relay/qnn/op/legalizations.py), dilate the data by the strides with
zeros, pad it by kernel - 1 - padding (plus output_padding at the bottom / right), flip the kernel
spatially and swap its I / O axes, then run an ordinary stride-1 grouped convolution.  The
reference's tests hold no literal vectors for this op, so parity with the reference itself stays
unpinned; this pins the oracle against a second derivation on grouped, strided
and output_padding cases.
"""
import numpy as np
import pytest

from oracle import qnn_ref as ref


def conv2d_transpose_topi(data, weight, za, zw, strides, padding, output_padding, groups):
    d = np.asarray(data).astype(np.int64) - int(za)
    w = np.asarray(weight).astype(np.int64)
    zw = np.asarray(zw, dtype=np.int64)
    w = w - (zw.reshape(1, -1, 1, 1) if zw.ndim else int(zw))
    n, c, h, wd = d.shape
    _, og, kh, kw = w.shape
    sh, sw = strides
    pt, pl, pb, pr = padding
    oph, opw = output_padding
    dil = np.zeros((n, c, (h - 1) * sh + 1, (wd - 1) * sw + 1), dtype=np.int64)
    dil[:, :, ::sh, ::sw] = d
    padded = np.pad(dil, ((0, 0), (0, 0), (kh - 1 - pt, kh - 1 - pb + oph), (kw - 1 - pl, kw - 1 - pr + opw)))
    cg = c // groups
    # kernel: flip, (C, O/g, KH, KW) -> per group (O/g, C/g, KH, KW)
    wf = w[:, :, ::-1, ::-1]
    oh = padded.shape[2] - kh + 1
    ow = padded.shape[3] - kw + 1
    out = np.zeros((n, og * groups, oh, ow), dtype=np.int64)
    for g in range(groups):
        wg = wf[g * cg:(g + 1) * cg].transpose(1, 0, 2, 3)  # (O/g, C/g, KH, KW)
        xg = padded[:, g * cg:(g + 1) * cg]
        for r in range(kh):
            for s in range(kw):
                out[:, g * og:(g + 1) * og] += np.einsum("nchw,oc->nohw", xg[:, :, r:r + oh, s:s + ow], wg[:, :, r, s])
    return ref.wrap_i32(out).astype(np.int32)


CASES = [
    # (N, C, H, W), (C, O/g, KH, KW), strides, padding (t, l, b, r), output_padding, groups
    ((2, 4, 5, 6), (4, 3, 3, 3), (1, 1), (1, 1, 1, 1), (0, 0), 1),
    ((1, 6, 4, 5), (6, 2, 3, 3), (2, 2), (1, 1, 1, 1), (1, 1), 1),
    ((2, 8, 3, 4), (8, 3, 4, 4), (2, 2), (1, 0, 2, 1), (0, 1), 2),
    ((1, 6, 5, 5), (6, 1, 3, 3), (2, 1), (0, 1, 0, 1), (1, 0), 6),      # depthwise, asymmetric strides
    ((1, 4, 3, 3), (4, 2, 5, 5), (3, 3), (2, 2, 2, 2), (2, 2), 2),
    ((1, 3, 4, 4), (3, 5, 1, 1), (2, 2), (0, 0, 0, 0), (1, 1), 1),      # 1x1 kernel: pure scatter
]


@pytest.mark.parametrize("dshape,wshape,strides,padding,opad,groups", CASES)
@pytest.mark.parametrize("dtype", ["int8", "uint8"])
def test_gather_oracle_equals_topi_form(dshape, wshape, strides, padding, opad, groups, dtype):
    rng = np.random.default_rng(sum(dshape) + sum(wshape))
    info = np.iinfo(dtype)
    x = rng.integers(info.min, int(info.max) + 1, size=dshape).astype(dtype)
    w = rng.integers(-128, 128, size=wshape).astype(np.int8)
    za = int(rng.integers(-5, 6)) + (128 if dtype == "uint8" else 0)
    for zw in (np.int32(0), np.int32(3), rng.integers(-4, 5, size=wshape[1] * 1).astype(np.int32)):
        if np.ndim(zw) and groups > 1:
            continue  # a vector kernel zero point runs along the weight's axis 1 (O / groups) only ungrouped
        got = ref.qnn_conv2d_transpose(x, w, za, zw, strides=strides, padding=padding, output_padding=opad,
                                       groups=groups)
        exp = conv2d_transpose_topi(x, w, za, zw, strides, padding, opad, groups)
        assert got.shape == exp.shape
        np.testing.assert_array_equal(got, exp)

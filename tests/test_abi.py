"""C-ABI library: loads without a GPU, exports every declared symbol, ctypes layouts match C,
and the host-side constant folding equals the oracle's restatement."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import qnn_ref as ref
from tachikoma_amd import _lib
from tachikoma_amd.relay.build_module import requantize_plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tachikoma.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tk_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) > 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)
    assert lib.tk_abi_version() == 1
    assert lib.tk_build_arch() == b"gfx950"


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "tachikoma.h"
#define P(T) printf(#T " %zu\n", sizeof(T));
#define O(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  P(tk_tensor) P(tk_requantize_attrs) P(tk_conv2d_attrs) P(tk_dense_attrs) P(tk_qnn_add_attrs)
  P(tk_pool2d_attrs) P(tk_block_attrs) P(tk_node) P(tk_array_meta) P(tk_trace_header) P(tk_postops_attrs)
  O(tk_postops_attrs, dst_zp) O(tk_postops_attrs, bias) O(tk_postops_attrs, o_scl)
  O(tk_tensor, shape) O(tk_tensor, byte_offset) O(tk_node, inputs) O(tk_node, n_outputs) O(tk_node, outputs) O(tk_node, ext)
  O(tk_node, attrs) O(tk_qnn_add_attrs, rhs) O(tk_qnn_add_attrs, lhs_upcast) O(tk_requantize_attrs, output_zero_point)
  O(tk_conv2d_attrs, kernel_zero_points) O(tk_array_meta, dtype)
  P(tk_qparams_attrs) P(tk_qnn_binary_attrs) P(tk_concat_attrs) P(tk_transpose_attrs)
  O(tk_qparams_attrs, zero_points) O(tk_qnn_binary_attrs, out) O(tk_qnn_binary_attrs, output_zero_point)
  O(tk_concat_attrs, rq)
  P(tk_leaky_relu_attrs) P(tk_conv2d_transpose_attrs) O(tk_leaky_relu_attrs, alpha_multiplier)
  O(tk_leaky_relu_attrs, zp_shift) O(tk_conv2d_transpose_attrs, kernel_zero_points) P(tk_simq_attrs)
  O(tk_simq_attrs, dtype_code) O(tk_simq_attrs, zero_points)
  P(tk_requantize_fp_attrs) P(tk_qnn_binary_fp_attrs) O(tk_requantize_fp_attrs, multiplier)
  O(tk_requantize_fp_attrs, input_zero_points) O(tk_requantize_fp_attrs, output_zero_point)
  O(tk_qnn_binary_fp_attrs, rhs) O(tk_qnn_binary_fp_attrs, out) O(tk_qnn_binary_fp_attrs, output_zero_point)
  return 0;
}
"""


def test_ctypes_layout_matches_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)]).decode().split("\n") if line)
    py = {
        "tk_tensor": ctypes.sizeof(_lib.tk_tensor), "tk_requantize_attrs": ctypes.sizeof(_lib.tk_requantize_attrs),
        "tk_conv2d_attrs": ctypes.sizeof(_lib.tk_conv2d_attrs), "tk_dense_attrs": ctypes.sizeof(_lib.tk_dense_attrs),
        "tk_qnn_add_attrs": ctypes.sizeof(_lib.tk_qnn_add_attrs), "tk_pool2d_attrs": ctypes.sizeof(_lib.tk_pool2d_attrs),
        "tk_node": ctypes.sizeof(_lib.tk_node), "tk_block_attrs": ctypes.sizeof(_lib.tk_block_attrs), "tk_array_meta": ctypes.sizeof(_lib.tk_array_meta),
        "tk_trace_header": 56, "tk_postops_attrs": ctypes.sizeof(_lib.tk_postops_attrs),
        "tk_postops_attrs.dst_zp": _lib.tk_postops_attrs.dst_zp.offset,
        "tk_postops_attrs.bias": _lib.tk_postops_attrs.bias.offset,
        "tk_postops_attrs.o_scl": _lib.tk_postops_attrs.o_scl.offset,
        "tk_tensor.shape": _lib.tk_tensor.shape.offset, "tk_tensor.byte_offset": _lib.tk_tensor.byte_offset.offset,
        "tk_node.inputs": _lib.tk_node.inputs.offset, "tk_node.n_outputs": _lib.tk_node.n_outputs.offset,
        "tk_node.outputs": _lib.tk_node.outputs.offset,
        "tk_node.ext": _lib.tk_node.ext.offset, "tk_node.attrs": _lib.tk_node.attrs.offset,
        "tk_qnn_add_attrs.rhs": _lib.tk_qnn_add_attrs.rhs.offset,
        "tk_qnn_add_attrs.lhs_upcast": _lib.tk_qnn_add_attrs.lhs_upcast.offset,
        "tk_requantize_attrs.output_zero_point": _lib.tk_requantize_attrs.output_zero_point.offset,
        "tk_conv2d_attrs.kernel_zero_points": _lib.tk_conv2d_attrs.kernel_zero_points.offset,
        "tk_array_meta.dtype": _lib.tk_array_meta.dtype.offset,
        "tk_qparams_attrs": ctypes.sizeof(_lib.tk_qparams_attrs),
        "tk_qnn_binary_attrs": ctypes.sizeof(_lib.tk_qnn_binary_attrs),
        "tk_concat_attrs": ctypes.sizeof(_lib.tk_concat_attrs),
        "tk_transpose_attrs": ctypes.sizeof(_lib.tk_transpose_attrs),
        "tk_qparams_attrs.zero_points": _lib.tk_qparams_attrs.zero_points.offset,
        "tk_qnn_binary_attrs.out": _lib.tk_qnn_binary_attrs.out.offset,
        "tk_qnn_binary_attrs.output_zero_point": _lib.tk_qnn_binary_attrs.output_zero_point.offset,
        "tk_concat_attrs.rq": _lib.tk_concat_attrs.rq.offset,
        "tk_leaky_relu_attrs": ctypes.sizeof(_lib.tk_leaky_relu_attrs),
        "tk_conv2d_transpose_attrs": ctypes.sizeof(_lib.tk_conv2d_transpose_attrs),
        "tk_leaky_relu_attrs.alpha_multiplier": _lib.tk_leaky_relu_attrs.alpha_multiplier.offset,
        "tk_leaky_relu_attrs.zp_shift": _lib.tk_leaky_relu_attrs.zp_shift.offset,
        "tk_conv2d_transpose_attrs.kernel_zero_points": _lib.tk_conv2d_transpose_attrs.kernel_zero_points.offset,
        "tk_simq_attrs": ctypes.sizeof(_lib.tk_simq_attrs),
        "tk_simq_attrs.dtype_code": _lib.tk_simq_attrs.dtype_code.offset,
        "tk_simq_attrs.zero_points": _lib.tk_simq_attrs.zero_points.offset,
        "tk_requantize_fp_attrs": ctypes.sizeof(_lib.tk_requantize_fp_attrs),
        "tk_qnn_binary_fp_attrs": ctypes.sizeof(_lib.tk_qnn_binary_fp_attrs),
        "tk_requantize_fp_attrs.multiplier": _lib.tk_requantize_fp_attrs.multiplier.offset,
        "tk_requantize_fp_attrs.input_zero_points": _lib.tk_requantize_fp_attrs.input_zero_points.offset,
        "tk_requantize_fp_attrs.output_zero_point": _lib.tk_requantize_fp_attrs.output_zero_point.offset,
        "tk_qnn_binary_fp_attrs.rhs": _lib.tk_qnn_binary_fp_attrs.rhs.offset,
        "tk_qnn_binary_fp_attrs.out": _lib.tk_qnn_binary_fp_attrs.out.offset,
        "tk_qnn_binary_fp_attrs.output_zero_point": _lib.tk_qnn_binary_fp_attrs.output_zero_point.offset,
    }
    for k, v in py.items():
        assert int(got[k]) == v, (k, got[k], v)


def test_fixed_point_multiplier_shift_matches_oracle():
    lib = _lib.load()
    rng = np.random.default_rng(0)
    vals = list(rng.uniform(1e-6, 10, size=2000)) + [0.0, 1.0, 0.5, 0.25, 1 / 3, 2.0, 3.0, 1e-9,
                                                      float(np.nextafter(1.0, 0.0)), 123456.789]
    vals += list(np.float64(rng.uniform(1e-4, 1, size=500).astype(np.float32)) /
                 np.float64(rng.uniform(1e-4, 1, size=500).astype(np.float32)))
    m, s = ctypes.c_int32(), ctypes.c_int32()
    for v in vals:
        _lib.check(lib.tk_fixed_point_multiplier_shift(float(v), ctypes.byref(m), ctypes.byref(s)))
        assert (m.value, s.value) == ref.get_fixed_point_multiplier_shift(float(v)), v


def test_requantize_prepare_modes():
    # equal scales skip FPM (requantize.cc:226); power of two → int32 path; per-axis always general
    assert requantize_plan(np.float32(0.5), np.float32(0.5), "UPWARD")[0] == _lib.TK_RQ_IDENTITY
    mode, ms, ss = requantize_plan(np.float32(1.0), np.float32(16.0), "UPWARD")
    assert mode == _lib.TK_RQ_TENSOR_POW2 and ms[0] == 1 << 30 and ss[0] == -3
    assert requantize_plan(np.float32(1.0), np.float32(16.0), "TONEAREST")[0] == _lib.TK_RQ_TENSOR_TONEAREST
    assert requantize_plan(np.float32(1.0), np.float32(3.0), "UPWARD")[0] == _lib.TK_RQ_TENSOR_UPWARD
    mode, ms, ss = requantize_plan(np.array([0.5, 0.5], np.float32), np.float32(0.5), "UPWARD")
    assert mode == _lib.TK_RQ_AXIS_UPWARD and list(ms) == [1 << 30, 1 << 30] and list(ss) == [1, 1]
    with pytest.raises(_lib.TachikomaError):
        requantize_plan(np.float32(1e-30), np.float32(1.0), "UPWARD")  # shift out of range


def test_no_gpu_needed_for_host_calls():
    # loading the library and host-only calls must not require a visible GPU
    lib = _lib.load()
    assert lib.tk_last_error() is not None


def _host_tensor(shape, code, bits, keep):
    """A tk_tensor descriptor with no data (host-only calls read shapes and dtypes)."""
    shp = (ctypes.c_int64 * len(shape))(*shape)
    keep.append(shp)
    t = _lib.tk_tensor()
    t.data = None
    t.ndim = len(shape)
    t.dtype.code, t.dtype.bits, t.dtype.lanes = code, bits, 1
    t.shape = shp
    t.strides = None
    return t


@pytest.mark.parametrize("n,c,h,o,k,want_pf", [
    (64, 64, 56, 256, 1, True),     # 56x56 expand: the persistent im2col kernel applies
    (64, 128, 28, 128, 3, True),    # 28x28 3x3 (taps of 64-byte stages)
    (64, 512, 7, 512, 3, False),    # 7x7: planes of <= 64 pixels take image-aligned tiles instead
])
def test_conv_block_algo_list(n, c, h, o, k, want_pf):
    # tk_conv2d_block_algos: im2col first, image-tile plans (16 + i), the persistent kernel (3, 4) last
    lib = _lib.load()
    keep = []
    x = _host_tensor((n, c, h, h), 0, 8, keep)
    w = _host_tensor((o, c, k, k), 0, 8, keep)
    a = _lib.tk_block_attrs()
    a.conv.strides[:] = [1, 1]
    p = k // 2
    a.conv.padding[:] = [p, p, p, p]
    a.conv.dilation[:] = [1, 1]
    a.conv.groups = 1
    a.requantize.mode = _lib.TK_RQ_AXIS_UPWARD
    a.requantize.axis = 1
    buf = (ctypes.c_int32 * 256)()
    cnt = lib.tk_conv2d_block_algos(ctypes.byref(x), ctypes.byref(w), ctypes.byref(a), buf, 256)
    assert 1 <= cnt <= 256
    algos = [int(buf[i]) for i in range(cnt)]
    assert algos[0] == 1
    has_pf = 3 in algos and 4 in algos
    assert has_pf == want_pf, algos
    if has_pf:
        assert algos[-2:] == [3, 4], algos
    assert all(x >= 16 for x in algos[1:len(algos) - (2 if has_pf else 0)]), algos
    # a short list keeps the head: the find step's first candidates
    short = (ctypes.c_int32 * 2)()
    assert lib.tk_conv2d_block_algos(ctypes.byref(x), ctypes.byref(w), ctypes.byref(a), short, 2) == cnt
    assert list(short) == algos[:2]


def test_conv_block_3x3_stage_widths():
    # 3x3 image-tile plans come with 32- and 64-channel K stages where the (padded) input channel
    # count divides by 64: a 512-channel 7x7 layer lists more plans than a 480-channel one (32 only)
    lib = _lib.load()

    def count(c):
        keep = []
        x = _host_tensor((64, c, 7, 7), 0, 8, keep)
        w = _host_tensor((512, c, 3, 3), 0, 8, keep)
        a = _lib.tk_block_attrs()
        a.conv.strides[:] = [1, 1]
        a.conv.padding[:] = [1, 1, 1, 1]
        a.conv.dilation[:] = [1, 1]
        a.conv.groups = 1
        a.requantize.mode = _lib.TK_RQ_AXIS_UPWARD
        a.requantize.axis = 1
        return lib.tk_conv2d_block_algos(ctypes.byref(x), ctypes.byref(w), ctypes.byref(a), None, 0)

    n512, n480 = count(512), count(480)
    assert n480 > 1 and n512 > n480, (n512, n480)


def test_conv_block_scratch_holds_split_partials():
    # a block's scratch holds the four partial records its split-K image-tile plans may write
    # (tk_conv_img.hip MODE 1 / 2); planes too large for image tiles reserve none of that
    lib = _lib.load()

    def scratch(c, h, o, k):
        keep = []
        x = _host_tensor((64, c, h, h), 0, 8, keep)
        w = _host_tensor((o, c, k, k), 0, 8, keep)
        a = _lib.tk_conv2d_attrs()
        a.strides[:] = [1, 1]
        p = k // 2
        a.padding[:] = [p, p, p, p]
        a.dilation[:] = [1, 1]
        a.groups = 1
        return lib.tk_conv2d_scratch_bytes(ctypes.byref(x), ctypes.byref(w), ctypes.byref(a), 1)

    assert scratch(512, 7, 512, 3) >= 4 * 64 * 512 * 49 * 4
    assert scratch(256, 14, 256, 3) >= 4 * 64 * 256 * 196 * 4
    assert scratch(1024, 7, 512, 1) >= 4 * 64 * 512 * 49 * 4
    assert scratch(64, 56, 256, 1) < 64 * 256 * 3136 * 4


def test_conv_block_algo_info():
    # every listed kernel has a description (the find step's report names its picks); unlisted fail
    lib = _lib.load()
    keep = []
    x = _host_tensor((64, 512, 7, 7), 0, 8, keep)
    w = _host_tensor((512, 512, 3, 3), 0, 8, keep)
    a = _lib.tk_block_attrs()
    a.conv.strides[:] = [1, 1]
    a.conv.padding[:] = [1, 1, 1, 1]
    a.conv.dilation[:] = [1, 1]
    a.conv.groups = 1
    a.requantize.mode = _lib.TK_RQ_AXIS_UPWARD
    a.requantize.axis = 1
    buf = (ctypes.c_int32 * 512)()
    cnt = lib.tk_conv2d_block_algos(ctypes.byref(x), ctypes.byref(w), ctypes.byref(a), buf, 512)
    descs = []
    for algo in list(buf)[:cnt]:
        s = ctypes.create_string_buffer(256)
        assert lib.tk_conv2d_block_algo_info(ctypes.byref(x), ctypes.byref(w), ctypes.byref(a), algo, s, 256) == 0
        descs.append(s.value.decode())
    assert descs[0].startswith("im2col")
    assert any(d.startswith("image tiles 3x3") and "split K" in d for d in descs), descs[:20]
    assert any(d.startswith("image tiles 3x3") and "split K" not in d for d in descs)
    s = ctypes.create_string_buffer(256)
    assert lib.tk_conv2d_block_algo_info(ctypes.byref(x), ctypes.byref(w), ctypes.byref(a), 16 + cnt + 5, s, 256) < 0

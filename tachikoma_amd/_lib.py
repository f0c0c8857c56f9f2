"""ctypes binding of ``libtachikoma.so`` (the C ABI declared in ``include/tachikoma.h``).

The library is built in-tree by ``tachikoma_amd/build.py``.  There is no CPU
fallback: if the library is missing every op raises ``TachikomaError``.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtachikoma.so")


class TachikomaError(RuntimeError):
    """Raised when a C-ABI call fails (carries ``tk_last_error()``)."""


# ---------------------------------------------------------------- structs (tachikoma.h)

class tk_device(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class tk_dtype(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class tk_tensor(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("device", tk_device),
        ("ndim", ctypes.c_int32),
        ("dtype", tk_dtype),
        ("shape", ctypes.POINTER(ctypes.c_int64)),
        ("strides", ctypes.POINTER(ctypes.c_int64)),
        ("byte_offset", ctypes.c_uint64),
    ]


class tk_requantize_attrs(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("axis", ctypes.c_int32),
        ("multiplier", ctypes.c_int32),
        ("shift", ctypes.c_int32),
        ("multipliers", ctypes.c_void_p),
        ("shifts", ctypes.c_void_p),
        ("input_zero_point", ctypes.c_int32),
        ("input_zero_points", ctypes.c_void_p),
        ("output_zero_point", ctypes.c_int32),
    ]


class tk_conv2d_attrs(ctypes.Structure):
    _fields_ = [
        ("strides", ctypes.c_int32 * 2),
        ("padding", ctypes.c_int32 * 4),
        ("dilation", ctypes.c_int32 * 2),
        ("groups", ctypes.c_int32),
        ("input_zero_point", ctypes.c_int32),
        ("kernel_zero_point", ctypes.c_int32),
        ("kernel_zero_points", ctypes.c_void_p),
    ]


class tk_dense_attrs(ctypes.Structure):
    _fields_ = [
        ("input_zero_point", ctypes.c_int32),
        ("kernel_zero_point", ctypes.c_int32),
        ("kernel_zero_points", ctypes.c_void_p),
    ]


class tk_qnn_add_attrs(ctypes.Structure):
    _fields_ = [
        ("lhs", tk_requantize_attrs),
        ("rhs", tk_requantize_attrs),
        ("output_zero_point", ctypes.c_int32),
        ("lhs_upcast", ctypes.c_int32),
        ("rhs_upcast", ctypes.c_int32),
    ]


class tk_block_attrs(ctypes.Structure):
    _fields_ = [
        ("conv", tk_conv2d_attrs),
        ("dense", tk_dense_attrs),
        ("requantize", tk_requantize_attrs),
        ("has_clip", ctypes.c_int32),
        ("clip_min", ctypes.c_int64),
        ("clip_max", ctypes.c_int64),
        ("has_add", ctypes.c_int32),
        ("block_is_rhs", ctypes.c_int32),
        ("residual", ctypes.POINTER(tk_tensor)),
        ("add", tk_qnn_add_attrs),
        ("algo", ctypes.c_int32),
    ]


class tk_add_block_attrs(ctypes.Structure):
    _fields_ = [
        ("add", tk_qnn_add_attrs),
        ("has_clip", ctypes.c_int32),
        ("clip_min", ctypes.c_int64),
        ("clip_max", ctypes.c_int64),
    ]


class tk_postops_attrs(ctypes.Structure):
    _fields_ = [
        ("axis", ctypes.c_int32),
        ("n_scales", ctypes.c_int32),
        ("clip_lo", ctypes.c_float),
        ("clip_hi", ctypes.c_float),
        ("act_scl", ctypes.c_float),
        ("sum_scl", ctypes.c_float),
        ("dst_zp", ctypes.c_float),
        ("bias", ctypes.c_void_p),
        ("o_scl", ctypes.c_void_p),
    ]


class tk_ewise_attrs(ctypes.Structure):
    _fields_ = [
        ("op", ctypes.c_int32),
        ("rhs_kind", ctypes.c_int32),
        ("scalar_f", ctypes.c_double),
        ("scalar_i", ctypes.c_int64),
        ("lo", ctypes.c_double),
        ("hi", ctypes.c_double),
        ("multiplier", ctypes.c_int32),
        ("shift", ctypes.c_int32),
    ]


TK_EW = {"add": 0, "multiply": 1, "left_shift": 2, "right_shift": 3, "round": 4, "clip": 5, "relu": 6,
         "fixed_point_multiply": 7}


class tk_pad_attrs(ctypes.Structure):
    _fields_ = [
        ("before", ctypes.c_int64 * 6),
        ("after", ctypes.c_int64 * 6),
        ("value_i", ctypes.c_int64),
        ("value_f", ctypes.c_double),
    ]


class tk_pool2d_attrs(ctypes.Structure):
    _fields_ = [
        ("pool_size", ctypes.c_int32 * 2),
        ("strides", ctypes.c_int32 * 2),
        ("padding", ctypes.c_int32 * 4),
        ("dilation", ctypes.c_int32 * 2),
        ("count_include_pad", ctypes.c_int32),
    ]


class tk_qparams_attrs(ctypes.Structure):
    _fields_ = [
        ("axis", ctypes.c_int32),
        ("scale", ctypes.c_float),
        ("scales", ctypes.c_void_p),
        ("zero_point", ctypes.c_int32),
        ("zero_points", ctypes.c_void_p),
    ]


class tk_qnn_binary_attrs(ctypes.Structure):
    _fields_ = [
        ("op", ctypes.c_int32),
        ("lhs", tk_requantize_attrs),
        ("rhs", tk_requantize_attrs),
        ("lhs_upcast", ctypes.c_int32),
        ("rhs_upcast", ctypes.c_int32),
        ("out", tk_requantize_attrs),
        ("output_zero_point", ctypes.c_int32),
    ]


TK_QB = {"qnn.add": 0, "qnn.subtract": 1, "qnn.mul": 2}
CONCAT_MAX = 8


class tk_concat_attrs(ctypes.Structure):
    _fields_ = [
        ("axis", ctypes.c_int32),
        ("n", ctypes.c_int32),
        ("requant", ctypes.c_int32 * CONCAT_MAX),
        ("rq", tk_requantize_attrs * CONCAT_MAX),
    ]


class tk_transpose_attrs(ctypes.Structure):
    _fields_ = [("ndim", ctypes.c_int32), ("perm", ctypes.c_int32 * 6)]


class tk_leaky_relu_attrs(ctypes.Structure):
    _fields_ = [
        ("rq", tk_requantize_attrs),
        ("upcast", ctypes.c_int32),
        ("input_zero_point", ctypes.c_int32),
        ("output_zero_point", ctypes.c_int32),
        ("alpha_multiplier", ctypes.c_int32),
        ("alpha_shift", ctypes.c_int32),
        ("zp_multiplier", ctypes.c_int32),
        ("zp_shift", ctypes.c_int32),
    ]


class tk_conv2d_transpose_attrs(ctypes.Structure):
    _fields_ = [
        ("strides", ctypes.c_int32 * 2),
        ("padding", ctypes.c_int32 * 4),
        ("output_padding", ctypes.c_int32 * 2),
        ("groups", ctypes.c_int32),
        ("input_zero_point", ctypes.c_int32),
        ("kernel_zero_point", ctypes.c_int32),
        ("kernel_zero_points", ctypes.c_void_p),
    ]


class tk_simq_attrs(ctypes.Structure):
    _fields_ = [
        ("axis", ctypes.c_int32),
        ("n_scales", ctypes.c_int32),
        ("n_zero_points", ctypes.c_int32),
        ("dtype_code", ctypes.c_void_p),
        ("scales", ctypes.c_void_p),
        ("zero_points", ctypes.c_void_p),
    ]


class tk_requantize_fp_attrs(ctypes.Structure):
    _fields_ = [
        ("bits", ctypes.c_int32),
        ("rounding", ctypes.c_int32),
        ("axis", ctypes.c_int32),
        ("scaled", ctypes.c_int32),
        ("multiplier", ctypes.c_double),
        ("multipliers", ctypes.c_void_p),
        ("input_zero_point", ctypes.c_int32),
        ("input_zero_points", ctypes.c_void_p),
        ("output_zero_point", ctypes.c_int32),
    ]


class tk_qnn_binary_fp_attrs(ctypes.Structure):
    _fields_ = [
        ("op", ctypes.c_int32),
        ("lhs", tk_requantize_fp_attrs),
        ("rhs", tk_requantize_fp_attrs),
        ("lhs_upcast", ctypes.c_int32),
        ("rhs_upcast", ctypes.c_int32),
        ("out", tk_requantize_fp_attrs),
        ("output_zero_point", ctypes.c_int32),
    ]


class _clip(ctypes.Structure):
    _fields_ = [("a_min", ctypes.c_int64), ("a_max", ctypes.c_int64)]


class _bias_add(ctypes.Structure):
    _fields_ = [("axis", ctypes.c_int32)]


class tk_node_attrs(ctypes.Union):
    _fields_ = [
        ("conv2d", tk_conv2d_attrs),
        ("dense", tk_dense_attrs),
        ("requantize", tk_requantize_attrs),
        ("qnn_add", tk_qnn_add_attrs),
        ("pool2d", tk_pool2d_attrs),
        ("block", tk_block_attrs),
        ("add_block", tk_add_block_attrs),
        ("postops", tk_postops_attrs),
        ("ewise", tk_ewise_attrs),
        ("pad", tk_pad_attrs),
        ("qparams", tk_qparams_attrs),
        ("qnn_binary", tk_qnn_binary_attrs),
        ("concat", tk_concat_attrs),
        ("transpose", tk_transpose_attrs),
        ("leaky_relu", tk_leaky_relu_attrs),
        ("conv2d_transpose", tk_conv2d_transpose_attrs),
        ("simq", tk_simq_attrs),
        ("requantize_fp", tk_requantize_fp_attrs),
        ("qnn_binary_fp", tk_qnn_binary_fp_attrs),
        ("clip", _clip),
        ("bias_add", _bias_add),
    ]


class tk_node(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("n_inputs", ctypes.c_int32),
        ("inputs", ctypes.POINTER(tk_tensor) * 8),
        ("n_outputs", ctypes.c_int32),
        ("outputs", ctypes.POINTER(tk_tensor) * 6),
        ("ext", ctypes.c_void_p * 5),
        ("attrs", tk_node_attrs),
    ]


class tk_array_meta(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char_p),
        ("ndim", ctypes.c_int32),
        ("shape", ctypes.POINTER(ctypes.c_int64)),
        ("dtype", tk_dtype),
    ]


# ---------------------------------------------------------------- constants
TK_DL_INT, TK_DL_UINT, TK_DL_FLOAT = 0, 1, 2
TK_DEV_CPU, TK_DEV_ROCM = 1, 10
TK_ROUND_UPWARD, TK_ROUND_TONEAREST = 0, 1
(TK_RQ_IDENTITY, TK_RQ_TENSOR_POW2, TK_RQ_TENSOR_UPWARD, TK_RQ_TENSOR_TONEAREST, TK_RQ_AXIS_UPWARD,
 TK_RQ_AXIS_TONEAREST) = range(6)
NODE_KINDS = {
    "qnn.conv2d": 1, "qnn.dense": 2, "qnn.requantize": 3, "nn.bias_add": 4, "clip": 5, "cast": 6,
    "qnn.add": 7, "nn.max_pool2d": 8, "nn.avg_pool2d": 9, "nn.global_avg_pool2d": 10, "copy": 11, "shadow": 12,
    "conv_block": 13, "dense_block": 14, "add_block": 15, "postops": 16,
    "ewise": 17, "conv2d_f32": 18, "dense_f32": 19, "nn.pad": 20,
    "qnn.quantize": 21, "qnn.dequantize": 22, "qnn_binary": 23, "qnn.concatenate": 24, "transpose": 25,
    "qnn.leaky_relu": 26, "lookup": 27, "qnn.batch_matmul": 28, "qnn.conv2d_transpose": 29,
    "qnn.simulated_quantize": 30, "qnn.simulated_dequantize": 31, "requantize_fp": 32, "qnn_binary_fp": 33,
}
MAX_NODE_INPUTS = 8
MAX_NODE_OUTPUTS = 6

# Every symbol declared in include/tachikoma.h, with its ctypes signature.
_VP, _I32, _I64, _F32, _F64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double
_PT = ctypes.POINTER(tk_tensor)
SIGNATURES = {
    "tk_last_error": (ctypes.c_char_p, []),
    "tk_abi_version": (ctypes.c_int, []),
    "tk_build_arch": (ctypes.c_char_p, []),
    "tk_build_info": (ctypes.c_char_p, []),
    "tk_fixed_point_multiplier_shift": (ctypes.c_int, [_F64, ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    "tk_requantize_prepare": (ctypes.c_int, [ctypes.POINTER(_F32), ctypes.c_int, _F32, ctypes.c_int,
                                             ctypes.POINTER(_I32), ctypes.POINTER(_I32), ctypes.POINTER(ctypes.c_int)]),
    "tk_conv2d_packed_weight_bytes": (_I64, [_PT, ctypes.c_int]),
    "tk_conv2d_pack_weight": (ctypes.c_int, [_PT, ctypes.c_int, _VP, _VP, _VP]),
    "tk_conv2d_shadow_bytes": (_I64, [_PT]),
    "tk_conv2d_scratch_bytes": (_I64, [_PT, _PT, ctypes.POINTER(tk_conv2d_attrs), ctypes.c_int]),
    "tk_conv2d_make_shadow": (ctypes.c_int, [_PT, _VP, _VP]),
    "tk_qnn_conv2d_prepared": (ctypes.c_int, [_PT, _VP, _PT, _VP, _VP, _PT, ctypes.POINTER(tk_conv2d_attrs), _VP,
                                              _VP]),
    "tk_qnn_conv2d_workspace_bytes": (_I64, [_PT, _PT, ctypes.POINTER(tk_conv2d_attrs)]),
    "tk_qnn_conv2d": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_conv2d_attrs), _VP, _VP]),
    "tk_qnn_dense_workspace_bytes": (_I64, [_PT, _PT]),
    "tk_qnn_dense": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_dense_attrs), _VP, _VP]),
    "tk_qnn_conv2d_block": (ctypes.c_int, [_PT, _VP, _PT, _VP, _VP, _PT, ctypes.POINTER(_PT), ctypes.c_int,
                                           ctypes.POINTER(tk_block_attrs), _VP, _VP, _VP]),
    "tk_qnn_dense_block": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(_PT), ctypes.c_int,
                                          ctypes.POINTER(tk_block_attrs), _VP, _VP]),
    "tk_requantize": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_requantize_attrs), _VP]),
    "tk_qnn_add": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_qnn_add_attrs), _VP]),
    "tk_qnn_add_block": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(_PT), ctypes.c_int,
                                        ctypes.POINTER(tk_add_block_attrs), _VP, _VP]),
    "tk_bias_add": (ctypes.c_int, [_PT, _PT, _PT, ctypes.c_int, _VP]),
    "tk_clip": (ctypes.c_int, [_PT, _PT, _I64, _I64, _VP]),
    "tk_cast": (ctypes.c_int, [_PT, _PT, _VP]),
    "tk_max_pool2d": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_pool2d_attrs), _VP]),
    "tk_max_pool2d_shadow": (ctypes.c_int, [_PT, _VP, _PT, ctypes.POINTER(tk_pool2d_attrs), _VP, _VP]),
    "tk_avg_pool2d": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_pool2d_attrs), _VP]),
    "tk_global_avg_pool2d": (ctypes.c_int, [_PT, _PT, _VP]),
    "tk_copy": (ctypes.c_int, [_PT, _PT, _VP]),
    "tk_pad": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_pad_attrs), _VP]),
    "tk_tachikoma_postops": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_postops_attrs), _VP]),
    "tk_ewise": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_ewise_attrs), _VP]),
    "tk_conv2d_f32": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_conv2d_attrs), _VP]),
    "tk_dense_f32": (ctypes.c_int, [_PT, _PT, _PT, _VP]),
    "tk_qnn_quantize": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_qparams_attrs), _VP]),
    "tk_qnn_dequantize": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_qparams_attrs), _VP]),
    "tk_qnn_binary": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_qnn_binary_attrs), _VP]),
    "tk_qnn_concatenate": (ctypes.c_int, [ctypes.POINTER(_PT), ctypes.c_int, _PT, ctypes.POINTER(tk_concat_attrs),
                                          _VP]),
    "tk_transpose": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_transpose_attrs), _VP]),
    "tk_qnn_leaky_relu": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_leaky_relu_attrs), _VP]),
    "tk_qnn_lookup": (ctypes.c_int, [_PT, _PT, _VP, _VP]),
    "tk_qnn_batch_matmul_workspace_bytes": (_I64, [_PT, _PT]),
    "tk_qnn_batch_matmul": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_dense_attrs), _VP, _VP]),
    "tk_qnn_conv2d_transpose": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_conv2d_transpose_attrs), _VP]),
    "tk_qnn_simulated_quantize": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_simq_attrs), _VP]),
    "tk_qnn_simulated_dequantize": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_simq_attrs), _VP]),
    "tk_requantize_fp": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_requantize_fp_attrs), _VP]),
    "tk_qnn_binary_fp": (ctypes.c_int, [_PT, _PT, _PT, ctypes.POINTER(tk_qnn_binary_fp_attrs), _VP]),
    "tk_find_scale_by_kl": (ctypes.c_int, [ctypes.POINTER(_I32), ctypes.POINTER(_F32), ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(_F32)]),
    "tk_module_create": (ctypes.c_int, [ctypes.POINTER(tk_node), ctypes.c_int, ctypes.POINTER(_VP)]),
    "tk_module_destroy": (ctypes.c_int, [_VP]),
    "tk_module_num_nodes": (ctypes.c_int, [_VP]),
    "tk_module_run": (ctypes.c_int, [_VP, _VP, _VP, ctypes.POINTER(_VP)]),
    "tk_module_wait_capture": (ctypes.c_int, [_VP, _VP]),
    "tk_module_run_range": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _VP]),
    "tk_module_run_profiled": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(_F32)]),
    "tk_module_set_profiling": (ctypes.c_int, [_VP, ctypes.c_int]),
    "tk_module_node_times": (ctypes.c_int, [_VP, ctypes.POINTER(_F32)]),
    "tk_module_run_graph": (ctypes.c_int, [_VP, _VP, _VP, ctypes.POINTER(_VP)]),
    "tk_module_set_graph_copies": (ctypes.c_int, [_VP, ctypes.c_int]),
    "tk_module_set_trace_chunks": (ctypes.c_int, [_VP, ctypes.c_int]),
    "tk_module_set_copy_trace": (ctypes.c_int, [_VP, ctypes.c_int]),
    "tk_module_copy_trace": (ctypes.c_int, [_VP, ctypes.POINTER(_F64), ctypes.c_int]),
    "tk_module_tune": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                      ctypes.POINTER(_F32)]),
    "tk_module_set_node_algo": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int]),
    "tk_conv2d_block_algos": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_block_attrs), ctypes.POINTER(ctypes.c_int32),
                                             ctypes.c_int]),
    "tk_conv2d_block_algo_info": (ctypes.c_int, [_PT, _PT, ctypes.POINTER(tk_block_attrs), ctypes.c_int,
                                                  ctypes.c_char_p, ctypes.c_int]),
    "tk_ndlist_layout": (_I64, [ctypes.POINTER(tk_array_meta), ctypes.c_int, ctypes.POINTER(_I64)]),
    "tk_ndlist_write_headers": (ctypes.c_int, [ctypes.POINTER(tk_array_meta), ctypes.c_int, _VP, _I64]),
    "tk_ndlist_parse": (ctypes.c_int, [_VP, _I64, ctypes.c_int, ctypes.POINTER(tk_array_meta), ctypes.POINTER(_I64),
                                       ctypes.POINTER(_I64), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "tk_trace_layout": (_I64, [ctypes.c_char_p, ctypes.POINTER(tk_array_meta), ctypes.c_int,
                               ctypes.POINTER(tk_array_meta), ctypes.c_int, ctypes.POINTER(_I64),
                               ctypes.POINTER(_I64)]),
    "tk_trace_write_headers": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(tk_array_meta), ctypes.c_int,
                                              ctypes.POINTER(tk_array_meta), ctypes.c_int, _VP, _I64]),
    "tk_write_file": (ctypes.c_int, [ctypes.c_char_p, _VP, _I64]),
    "tk_digest_bytes": (ctypes.c_int, [_VP, _I64, _VP, _VP]),
}

_LIB: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the HIP library (fails loudly: there is no fallback path).

    The library must have been built from the sources of this tree: its ``tk_build_info()``
    (the source digest compiled in by build.py) is compared with the digest of the in-tree
    sources, and a stale library is refused.  ``TK_LIB_PATH`` substitutes the ablation build
    of the same sources (A/B kernel timing in tools/, one process per build on one box); it
    is announced on stderr and reported by ``build_info()``; with ``TK_LIB_ANY_SOURCES=1`` it may
    be a build of other sources (A/B of two versions)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    override = os.environ.get("TK_LIB_PATH")
    path = override or path
    if not os.path.exists(path):
        raise TachikomaError(
            f"{path} not found: build it with `python tachikoma_amd/build.py` "
            "(the engine has no CPU fallback)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    from .build import source_hash
    built = lib.tk_build_info().decode()
    try:
        want = source_hash()
    except OSError:
        # a deployment that ships the library without its sources: nothing to compare with
        want = None
    # TK_LIB_ANY_SOURCES=1 (with TK_LIB_PATH only): A/B timing of another source version's build
    # on the same box (the C ABI and the planner's algo numbering must be unchanged between them)
    any_src = bool(override) and os.environ.get("TK_LIB_ANY_SOURCES") == "1"
    if want is not None and built.split("+")[0] != want and not any_src:
        raise TachikomaError(
            f"{path} was built from other sources (library {built}, tree {want}): rebuild it with "
            "`python tachikoma_amd/build.py`")
    if override:
        import sys
        sys.stderr.write(f"[tachikoma] TK_LIB_PATH: using {path} ({built})\n")
    _LIB = lib
    return lib


def build_info() -> str:
    """Source digest (and build flavour) of the loaded library."""
    return load().tk_build_info().decode()


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().tk_last_error().decode(errors="replace")
        raise TachikomaError(f"{what or 'tachikoma call'} failed ({rc}): {msg}")


# ---------------------------------------------------------------- dtype helpers
_DT = {
    "int8": (TK_DL_INT, 8), "uint8": (TK_DL_UINT, 8), "int16": (TK_DL_INT, 16), "uint16": (TK_DL_UINT, 16),
    "int32": (TK_DL_INT, 32), "uint32": (TK_DL_UINT, 32), "int64": (TK_DL_INT, 64), "uint64": (TK_DL_UINT, 64),
    "float32": (TK_DL_FLOAT, 32), "float64": (TK_DL_FLOAT, 64),
}


def dtype_struct(dtype: str) -> tk_dtype:
    code, bits = _DT[str(np.dtype(dtype))]
    return tk_dtype(code, bits, 1)


def dtype_name(d: tk_dtype) -> str:
    for k, (c, b) in _DT.items():
        if c == d.code and b == d.bits:
            return k
    raise TachikomaError(f"unknown dtype code={d.code} bits={d.bits}")


class TensorRef:
    """A tk_tensor describing device (or host) memory owned elsewhere; keeps its shape alive."""

    def __init__(self, data_ptr: int, shape, dtype: str, device_type: int = TK_DEV_ROCM, device_id: int = 0):
        self.shape_arr = (ctypes.c_int64 * max(1, len(shape)))(*[int(s) for s in shape])
        self.struct = tk_tensor()
        self.struct.data = ctypes.c_void_p(int(data_ptr))
        self.struct.device = tk_device(device_type, device_id)
        self.struct.ndim = len(shape)
        self.struct.dtype = dtype_struct(dtype)
        self.struct.shape = ctypes.cast(self.shape_arr, ctypes.POINTER(ctypes.c_int64))
        self.struct.strides = None
        self.struct.byte_offset = 0
        self.shape = tuple(int(s) for s in shape)
        self.dtype = str(np.dtype(dtype))

    @property
    def ptr(self):
        return ctypes.pointer(self.struct)

    @staticmethod
    def from_torch(t) -> "TensorRef":
        import torch
        assert t.is_contiguous(), "tensors must be compact"
        dev = TK_DEV_ROCM if t.is_cuda else TK_DEV_CPU
        return TensorRef(t.data_ptr(), tuple(t.shape), str(t.dtype).replace("torch.", ""), dev,
                         t.device.index or 0 if t.is_cuda else 0)


def stream_handle(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)

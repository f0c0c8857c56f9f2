"""Helpers that call single C-ABI ops on the GPU with numpy inputs (used by -m gpu tests)."""
import ctypes

import numpy as np

from tachikoma_amd import _lib
from tachikoma_amd.relay.build_module import requantize_plan


def _torch():
    import torch
    return torch


def dev(x: np.ndarray):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def empty(shape, dtype):
    torch = _torch()
    from tachikoma_amd.relay.device_module import torch_dtype
    return torch.empty(tuple(shape), dtype=torch_dtype(str(np.dtype(dtype))), device="cuda")


def ref(t):
    return _lib.TensorRef.from_torch(t)


def _sync_check(rc, what):
    _lib.check(rc, what)
    _torch().cuda.synchronize()


def stream():
    return ctypes.c_void_p(_lib.stream_handle())


def conv2d(x, w, za, zw, strides=(1, 1), padding=(0, 0, 0, 0), dilation=(1, 1), groups=1, zw_vec=None):
    lib = _lib.load()
    n, c, h, wd = x.shape
    o, cg, kh, kw = w.shape
    pt, pl, pb, pr = padding
    oh = (h + pt + pb - dilation[0] * (kh - 1) - 1) // strides[0] + 1
    ow = (wd + pl + pr - dilation[1] * (kw - 1) - 1) // strides[1] + 1
    xd, wdv = dev(x), dev(w)
    out = empty((n, o, oh, ow), "int32")
    a = _lib.tk_conv2d_attrs()
    a.strides[:] = list(strides)
    a.padding[:] = list(padding)
    a.dilation[:] = list(dilation)
    a.groups = groups
    a.input_zero_point = int(za)
    a.kernel_zero_point = int(zw)
    keep = None
    if zw_vec is not None:
        keep = dev(np.asarray(zw_vec, np.int32))
        a.kernel_zero_points = keep.data_ptr()
    rx, rw, ro = ref(xd), ref(wdv), ref(out)
    ws_bytes = lib.tk_qnn_conv2d_workspace_bytes(rx.ptr, rw.ptr, ctypes.byref(a))
    assert ws_bytes >= 0
    ws = empty((max(ws_bytes, 16),), "uint8")
    _sync_check(lib.tk_qnn_conv2d(rx.ptr, rw.ptr, ro.ptr, ctypes.byref(a), ctypes.c_void_p(ws.data_ptr()), stream()),
                "tk_qnn_conv2d")
    return out.cpu().numpy()


def dense(x, w, za, zw, zw_vec=None):
    lib = _lib.load()
    xd, wdv = dev(x), dev(w)
    out = empty((x.shape[0], w.shape[0]), "int32")
    a = _lib.tk_dense_attrs()
    a.input_zero_point = int(za)
    a.kernel_zero_point = int(zw)
    keep = None
    if zw_vec is not None:
        keep = dev(np.asarray(zw_vec, np.int32))
        a.kernel_zero_points = keep.data_ptr()
    rx, rw, ro = ref(xd), ref(wdv), ref(out)
    ws_bytes = lib.tk_qnn_dense_workspace_bytes(rx.ptr, rw.ptr)
    ws = empty((max(ws_bytes, 16),), "uint8")
    _sync_check(lib.tk_qnn_dense(rx.ptr, rw.ptr, ro.ptr, ctypes.byref(a), ctypes.c_void_p(ws.data_ptr()), stream()),
                "tk_qnn_dense")
    return out.cpu().numpy()


def requantize(x, input_scale, input_zero_point, output_scale, output_zero_point, axis=-1, rounding="UPWARD",
               out_dtype="int8"):
    lib = _lib.load()
    mode, ms, ss = requantize_plan(input_scale, output_scale, rounding)
    xd = dev(x)
    out = empty(x.shape, out_dtype)
    a = _lib.tk_requantize_attrs()
    a.mode = mode
    nd = x.ndim
    a.axis = (axis if axis >= 0 else nd + axis) if nd else 0
    keep = []
    if mode >= _lib.TK_RQ_AXIS_UPWARD:
        m_d, s_d = dev(ms), dev(ss)
        keep += [m_d, s_d]
        a.multipliers = m_d.data_ptr()
        a.shifts = s_d.data_ptr()
    else:
        a.multiplier = int(ms[0])
        a.shift = int(ss[0])
    zpi = np.asarray(input_zero_point)
    if zpi.ndim == 0:
        a.input_zero_point = int(zpi)
    else:
        z = dev(zpi.astype(np.int32))
        keep.append(z)
        a.input_zero_points = z.data_ptr()
    a.output_zero_point = int(output_zero_point)
    rx, ro = ref(xd), ref(out)
    _sync_check(lib.tk_requantize(rx.ptr, ro.ptr, ctypes.byref(a), stream()), "tk_requantize")
    return out.cpu().numpy()


def qnn_add(lhs, rhs, ls, lz, rs, rz, os_, oz):
    lib = _lib.load()
    a = _lib.tk_qnn_add_attrs()
    _add_attrs(a, ls, lz, rs, rz, os_, oz)
    ld, rd = dev(lhs), dev(rhs)
    out = empty(lhs.shape, str(lhs.dtype))
    _sync_check(lib.tk_qnn_add(ref(ld).ptr, ref(rd).ptr, ref(out).ptr, ctypes.byref(a), stream()), "tk_qnn_add")
    return out.cpu().numpy()


def _add_attrs(a, ls, lz, rs, rz, os_, oz):
    for side, s, z in (("lhs", ls, lz), ("rhs", rs, rz)):
        r = getattr(a, side)
        up = np.float32(s).tobytes() == np.float32(os_).tobytes() and int(z) == int(oz)
        setattr(a, f"{side}_upcast", int(up))
        if not up:
            mode, ms, ss = requantize_plan(np.float32(s), np.float32(os_), "UPWARD")
            r.mode, r.multiplier, r.shift = mode, int(ms[0]), int(ss[0])
        r.input_zero_point = int(z)
        r.output_zero_point = int(oz)
    a.output_zero_point = int(oz)


def qnn_add_block(lhs, rhs, ls, lz, rs, rz, os_, oz, clip=None, want_shadow=False):
    """Fused qnn.add [-> clip] through tk_qnn_add_block; returns [add, (clip), (shadow)]."""
    lib = _lib.load()
    a = _lib.tk_add_block_attrs()
    _add_attrs(a.add, ls, lz, rs, rz, os_, oz)
    if clip is not None:
        a.has_clip = 1
        a.clip_min, a.clip_max = clip
    ld, rd = dev(lhs), dev(rhs)
    outs = [empty(lhs.shape, str(lhs.dtype))]
    if clip is not None:
        outs.append(empty(lhs.shape, str(lhs.dtype)))
    shadow = None
    if want_shadow:
        torch = _torch()
        n, c, h, w = lhs.shape
        # poisoned: the kernel must write every byte incl. the padded channels
        shadow = torch.full(((c + 15) // 16, n * h * w, 16), 0x5A, dtype=torch.uint8, device="cuda")
    refs = [ref(t) for t in outs]
    arr = (ctypes.POINTER(_lib.tk_tensor) * len(refs))(*[r.ptr for r in refs])
    _sync_check(lib.tk_qnn_add_block(ref(ld).ptr, ref(rd).ptr, arr, len(refs), ctypes.byref(a),
                                     ctypes.c_void_p(shadow.data_ptr()) if shadow is not None else None, stream()),
                "tk_qnn_add_block")
    res = [t.cpu().numpy() for t in outs]
    if shadow is not None:
        res.append(shadow.cpu().numpy())
    return res


def unary(name, x, out_dtype=None, *extra):
    lib = _lib.load()
    xd = dev(x)
    out = empty(x.shape, out_dtype or str(x.dtype))
    fn = getattr(lib, name)
    _sync_check(fn(ref(xd).ptr, ref(out).ptr, *extra, stream()), name)
    return out.cpu().numpy()


def bias_add(x, b, axis=1):
    lib = _lib.load()
    xd, bd = dev(x), dev(b)
    out = empty(x.shape, str(x.dtype))
    _sync_check(lib.tk_bias_add(ref(xd).ptr, ref(bd).ptr, ref(out).ptr, axis, stream()), "tk_bias_add")
    return out.cpu().numpy()


def pool(name, x, pool_size, strides, padding, dilation=(1, 1), count_include_pad=False):
    lib = _lib.load()
    n, c, h, w = x.shape
    kh, kw = pool_size
    oh = (h + padding[0] + padding[2] - dilation[0] * (kh - 1) - 1) // strides[0] + 1
    ow = (w + padding[1] + padding[3] - dilation[1] * (kw - 1) - 1) // strides[1] + 1
    a = _lib.tk_pool2d_attrs()
    a.pool_size[:] = list(pool_size)
    a.strides[:] = list(strides)
    a.padding[:] = list(padding)
    a.dilation[:] = list(dilation)
    a.count_include_pad = int(count_include_pad)
    xd = dev(x)
    out = empty((n, c, oh, ow), str(x.dtype))
    _sync_check(getattr(lib, name)(ref(xd).ptr, ref(out).ptr, ctypes.byref(a), stream()), name)
    return out.cpu().numpy()


def max_pool_shadow(x, pool_size, strides, padding, dilation=(1, 1)):
    """tk_max_pool2d_shadow: input read from its conv shadow; returns (record, output shadow)."""
    lib = _lib.load()
    n, c, h, w = x.shape
    kh, kw = pool_size
    oh = (h + padding[0] + padding[2] - dilation[0] * (kh - 1) - 1) // strides[0] + 1
    ow = (w + padding[1] + padding[3] - dilation[1] * (kw - 1) - 1) // strides[1] + 1
    a = _lib.tk_pool2d_attrs()
    a.pool_size[:] = list(pool_size)
    a.strides[:] = list(strides)
    a.padding[:] = list(padding)
    a.dilation[:] = list(dilation)
    xd = dev(x)
    rx = ref(xd)
    torch = _torch()
    sin = torch.empty(lib.tk_conv2d_shadow_bytes(rx.ptr), dtype=torch.uint8, device="cuda")
    _lib.check(lib.tk_conv2d_make_shadow(rx.ptr, ctypes.c_void_p(sin.data_ptr()), stream()))
    out = empty((n, c, oh, ow), str(x.dtype))
    sout = torch.full(((c + 15) // 16, n * oh * ow, 16), 0x5A, dtype=torch.uint8, device="cuda")
    _sync_check(lib.tk_max_pool2d_shadow(rx.ptr, ctypes.c_void_p(sin.data_ptr()), ref(out).ptr, ctypes.byref(a),
                                         ctypes.c_void_p(sout.data_ptr()), stream()), "tk_max_pool2d_shadow")
    return out.cpu().numpy(), sout.cpu().numpy()


def global_avg_pool(x):
    lib = _lib.load()
    xd = dev(x)
    out = empty((x.shape[0], x.shape[1], 1, 1), str(x.dtype))
    _sync_check(lib.tk_global_avg_pool2d(ref(xd).ptr, ref(out).ptr, stream()), "tk_global_avg_pool2d")
    return out.cpu().numpy()


def _rq_attrs(r, keep, input_scale, output_scale, output_zero_point, rounding="UPWARD", axis=1):
    mode, ms, ss = requantize_plan(input_scale, output_scale, rounding)
    r.mode = mode
    r.axis = axis
    if mode >= _lib.TK_RQ_AXIS_UPWARD:
        m_d, s_d = dev(ms), dev(ss)
        keep += [m_d, s_d]
        r.multipliers = m_d.data_ptr()
        r.shifts = s_d.data_ptr()
    else:
        r.multiplier, r.shift = int(ms[0]), int(ss[0])
    r.output_zero_point = int(output_zero_point)


def conv2d_block(x, w, bias, za, zw, s_in, s_out, zp_out, clip=None, strides=(1, 1), padding=(0, 0, 0, 0),
                 dilation=(1, 1), groups=1, out_dtype="int8", want_shadow=False, residual=None, add_params=None,
                 block_is_rhs=False, rounding="UPWARD", algo=0, algos_only=False, zw_vec=None):
    """Fused conv -> bias_add -> requantize(axis 1) [-> qnn.add(., residual)] [-> clip] through
    tk_qnn_conv2d_block.  add_params = (ls, lz, rs, rz, os, oz) of the qnn.add (lhs = the block's
    requantize output unless block_is_rhs).  algo: tk_block_attrs.algo; algos_only: return the
    block's kernel list (tk_conv2d_block_algos) instead of running it."""
    lib = _lib.load()
    n, c, h, wd = x.shape
    o = w.shape[0]
    kh, kw = w.shape[2], w.shape[3]
    pt, pl, pb, pr = padding
    oh = (h + pt + pb - dilation[0] * (kh - 1) - 1) // strides[0] + 1
    ow = (wd + pl + pr - dilation[1] * (kw - 1) - 1) // strides[1] + 1
    xd, wdv, bd = dev(x), dev(w), dev(bias)
    outs = [empty((n, o, oh, ow), "int32"), empty((n, o, oh, ow), "int32"), empty((n, o, oh, ow), out_dtype)]
    if residual is not None:
        outs.append(empty((n, o, oh, ow), out_dtype))
    if clip is not None:
        outs.append(empty((n, o, oh, ow), out_dtype))
    a = _lib.tk_block_attrs()
    a.conv.strides[:] = list(strides)
    a.conv.padding[:] = list(padding)
    a.conv.dilation[:] = list(dilation)
    a.conv.groups = groups
    a.conv.input_zero_point = int(za)
    a.conv.kernel_zero_point = int(zw)
    keep = []
    if zw_vec is not None:  # per-output-channel kernel zero points
        keep.append(dev(np.asarray(zw_vec, np.int32)))
        a.conv.kernel_zero_points = keep[-1].data_ptr()
    _rq_attrs(a.requantize, keep, s_in, s_out, zp_out, rounding=rounding)
    if clip is not None:
        a.has_clip = 1
        a.clip_min, a.clip_max = clip
    res_keep = None
    if residual is not None:
        res_keep = dev(residual)
        res_ref = ref(res_keep)
        a.has_add = 1
        a.block_is_rhs = int(block_is_rhs)
        a.residual = res_ref.ptr
        _add_attrs(a.add, *add_params)
    a.algo = int(algo)
    rx, rw, rb = ref(xd), ref(wdv), ref(bd)
    if algos_only:
        buf = (ctypes.c_int32 * 256)()
        cnt = lib.tk_conv2d_block_algos(rx.ptr, rw.ptr, ctypes.byref(a), buf, 256)
        _lib.check(min(cnt, 0), "tk_conv2d_block_algos")
        assert cnt <= 256
        return [int(buf[i]) for i in range(cnt)]
    ws_bytes = lib.tk_qnn_conv2d_workspace_bytes(rx.ptr, rw.ptr, ctypes.byref(a.conv))
    shadow = packed = sums = patch = shadow_out = None
    st = stream()
    if ws_bytes > 0:
        shadow = empty((lib.tk_conv2d_shadow_bytes(rx.ptr),), "uint8")
        packed = empty((lib.tk_conv2d_packed_weight_bytes(rw.ptr, 1),), "uint8")
        sums = empty((((o + 127) // 128) * 128,), "int32")
        sb = lib.tk_conv2d_scratch_bytes(rx.ptr, rw.ptr, ctypes.byref(a.conv), 1)
        assert sb >= 0
        patch = empty((max(sb, 16),), "uint8")
        _lib.check(lib.tk_conv2d_make_shadow(rx.ptr, ctypes.c_void_p(shadow.data_ptr()), st))
        _lib.check(lib.tk_conv2d_pack_weight(rw.ptr, 1, ctypes.c_void_p(packed.data_ptr()),
                                             ctypes.c_void_p(sums.data_ptr()), st))
    if want_shadow:
        import torch
        cpad = (o + 15) // 16 * 16
        # poisoned: the kernel must write every byte incl. the padded channels
        shadow_out = torch.full((cpad // 16, n * oh * ow, 16), 0x5A, dtype=torch.uint8, device="cuda")
    refs = [ref(t) for t in outs]
    arr = (ctypes.POINTER(_lib.tk_tensor) * len(refs))(*[r.ptr for r in refs])
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    _sync_check(lib.tk_qnn_conv2d_block(rx.ptr, ptr(shadow), rw.ptr, ptr(packed), ptr(sums), rb.ptr, arr, len(refs),
                                        ctypes.byref(a), ptr(patch), ptr(shadow_out), st), "tk_qnn_conv2d_block")
    res = [t.cpu().numpy() for t in outs]
    if want_shadow:
        res.append(shadow_out.cpu().numpy())
    return res

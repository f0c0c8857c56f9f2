"""Microbenchmark of the fused residual kernel (tk_qnn_add_block) on the ResNet-50
stage shapes at batch 64, with and without the clip record / shadow, next to a
torch int8 add (2 reads + 1 write) as a streaming reference.  GPU only."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tachikoma_amd import _lib  # noqa: E402
sys.path.insert(0, "tests")
import tk_gpu  # noqa: E402


def timeit(fn, iters=20):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    lib = _lib.load()
    st = ctypes.c_void_p(_lib.stream_handle())
    for c, hw in ((256, 56), (512, 28), (1024, 14), (2048, 7)):
        shape = (64, c, hw, hw)
        n_el = int(np.prod(shape))
        a = torch.randint(-128, 128, shape, dtype=torch.int8, device="cuda")
        b = torch.randint(-128, 128, shape, dtype=torch.int8, device="cuda")
        outs = [torch.empty_like(a), torch.empty_like(a)]
        shadow = torch.empty(((c + 15) // 16) * 64 * hw * hw * 16, dtype=torch.uint8, device="cuda")
        at = _lib.tk_add_block_attrs()
        tk_gpu._add_attrs(at.add, 0.05, 3, 0.07, -2, 0.09, 1)
        refs = [_lib.TensorRef.from_torch(t) for t in (a, b) + tuple(outs)]
        res = []
        for name, n_outs, clip, sh in (("add", 1, 0, None), ("add+clip", 2, 1, None),
                                       ("add+clip+shadow", 2, 1, shadow)):
            at.has_clip = clip
            at.clip_min, at.clip_max = 1, 127
            arr = (ctypes.POINTER(_lib.tk_tensor) * n_outs)(*[r.ptr for r in refs[2:2 + n_outs]])
            shp = ctypes.c_void_p(sh.data_ptr()) if sh is not None else None
            us = timeit(lambda: _lib.check(lib.tk_qnn_add_block(refs[0].ptr, refs[1].ptr, arr, n_outs,
                                                                 ctypes.byref(at), shp, st)))
            nbytes = n_el * (2 + n_outs + (1 if sh is not None else 0))
            res.append(f"{name} {us:6.1f} us {nbytes / us / 1e3:5.0f} GB/s")
        us = timeit(lambda: torch.add(a, b, out=outs[0]))
        res.append(f"torch add {us:6.1f} us {3 * n_el / us / 1e3:5.0f} GB/s")
        print(f"{c}x{hw}x{hw}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()

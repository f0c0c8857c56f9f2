"""Microbenchmark of the fused conv block kernel on representative ResNet-50 layer shapes
(batch 64).  Prints time per call, algorithmic GB/s and TOPS.  GPU only."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tachikoma_amd import _lib  # noqa: E402
from tachikoma_amd.relay.build_module import requantize_plan  # noqa: E402

SHAPES = [  # name, C, H, O, K, stride, pad
    ("stem 3->64 k7 s2", 3, 224, 64, 7, 2, 3),
    ("1x1 64->256 56", 64, 56, 256, 1, 1, 0),
    ("1x1 256->64 56", 256, 56, 64, 1, 1, 0),
    ("3x3 64->64 56", 64, 56, 64, 3, 1, 1),
    ("3x3 128->128 28", 128, 28, 128, 3, 1, 1),
    ("3x3 256->256 14", 256, 14, 256, 3, 1, 1),
    ("1x1 1024->256 14", 1024, 14, 256, 1, 1, 0),
    ("1x1 256->1024 14", 256, 14, 1024, 1, 1, 0),
    ("ds 1x1 512->1024 s2 14", 512, 28, 1024, 1, 2, 0),
    ("1x1 512->256 s2 14", 512, 28, 256, 1, 2, 0),
    ("3x3 512->512 7", 512, 7, 512, 3, 1, 1),
    ("1x1 512->2048 7", 512, 7, 2048, 1, 1, 0),
    ("1x1 2048->512 7", 2048, 7, 512, 1, 1, 0),
    # expand layers with the fused residual join (qnn.add -> clip), as in every bottleneck
    ("1x1 128->512 28", 128, 28, 512, 1, 1, 0),
    ("res 1x1 64->256 56", 64, 56, 256, 1, 1, 0),
    ("res 1x1 128->512 28", 128, 28, 512, 1, 1, 0),
    ("res 1x1 256->1024 14", 256, 14, 1024, 1, 1, 0),
    ("res 1x1 512->2048 7", 512, 7, 2048, 1, 1, 0),
]


def main(batch=64, iters=20, configs=None, reps=3, only=None, rotate=1, marker=False, rotate_res=1):
    """configs: list of env-var dicts (TK_ABLATE / TK_NT are read per launch); each layer is
    timed for every config, interleaved `reps` times, and the minimum is reported."""
    import os
    configs = configs or [{}]
    lib = _lib.load()
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    tot = [0.0] * len(configs)
    for name, C, H, O, K, S, P in SHAPES:
        if only and not any(o in name for o in only.split(",")):
            continue
        OH = (H + 2 * P - K) // S + 1
        x = torch.from_numpy(rng.integers(-128, 128, size=(batch, C, H, H)).astype(np.int8)).to(dev)
        w = torch.from_numpy(rng.integers(-128, 128, size=(O, C, K, K)).astype(np.int8)).to(dev)
        b = torch.from_numpy(rng.integers(-2**14, 2**14, size=O).astype(np.int32)).to(dev)
        res = name.startswith("res ")
        # rotate > 1: that many output sets, used in turn (fresh pages / cold caches per call,
        # like the network, where every record has its own buffer)
        out_sets = [[torch.empty((batch, O, OH, OH), dtype=t, device=dev)
                     for t in (torch.int32, torch.int32, torch.int8) + ((torch.int8,) if res else ()) + (torch.int8,)]
                    for _ in range(rotate)]
        outs = out_sets[0]
        a = _lib.tk_block_attrs()
        a.conv.strides[:] = [S, S]
        a.conv.padding[:] = [P] * 4
        a.conv.dilation[:] = [1, 1]
        a.conv.groups = 1
        a.conv.input_zero_point = 3
        mode, ms, ss = requantize_plan(rng.uniform(1e-5, 1e-4, size=O).astype(np.float32), np.float32(0.05), "UPWARD")
        md, sd = torch.from_numpy(ms).to(dev), torch.from_numpy(ss).to(dev)
        a.requantize.mode, a.requantize.axis = mode, 1
        a.requantize.multipliers, a.requantize.shifts = md.data_ptr(), sd.data_ptr()
        a.requantize.output_zero_point = 2
        a.has_clip, a.clip_min, a.clip_max = 1, 2, 127
        a.algo = int(os.environ.get("TK_BB_ALGO", "0"))  # a tk_conv2d_block_algos entry (0: the library's choice)
        keep = []
        res_refs = []
        if res:
            # rotate_res > 1: that many residual operands in turn (in the network the residual is a
            # record written several kernels earlier, no longer in the MALL; here it would be)
            for _ in range(rotate_res):
                resid = torch.from_numpy(rng.integers(-128, 128, size=(batch, O, OH, OH)).astype(np.int8)).to(dev)
                rr = _lib.TensorRef.from_torch(resid)
                keep += [resid, rr]
                res_refs.append(rr)
            a.has_add, a.block_is_rhs, a.residual = 1, 0, res_refs[0].ptr
            for side, ratio in ((a.add.lhs, 0.71), (a.add.rhs, 1.37)):
                m_, ms_, ss_ = requantize_plan(np.float32(ratio * 0.05), np.float32(0.05), "UPWARD")
                side.mode, side.axis = m_, -1
                side.multiplier, side.shift = int(ms_[0]), int(ss_[0])
                side.input_zero_point, side.output_zero_point = 1, 3
            a.add.output_zero_point = 3
        rx, rw, rb = [_lib.TensorRef.from_torch(t) for t in (x, w, b)]
        ref_sets = [[_lib.TensorRef.from_torch(t) for t in o] for o in out_sets]
        arrs = [(ctypes.POINTER(_lib.tk_tensor) * len(r))(*[x.ptr for x in r]) for r in ref_sets]
        refs = ref_sets[0]
        turn = [0]
        st = ctypes.c_void_p(_lib.stream_handle())
        shadow = torch.empty(lib.tk_conv2d_shadow_bytes(rx.ptr), dtype=torch.uint8, device=dev)
        packed = torch.empty(lib.tk_conv2d_packed_weight_bytes(rw.ptr, 1), dtype=torch.uint8, device=dev)
        sums = torch.empty(((O + 127) // 128) * 128, dtype=torch.int32, device=dev)
        sb = lib.tk_conv2d_scratch_bytes(rx.ptr, rw.ptr, ctypes.byref(a.conv), 1)
        scratch = torch.empty(max(sb, 16), dtype=torch.uint8, device=dev)
        sh_out = torch.zeros(batch * OH * OH * ((O + 15) // 16 * 16), dtype=torch.uint8, device=dev)
        _lib.check(lib.tk_conv2d_make_shadow(rx.ptr, ctypes.c_void_p(shadow.data_ptr()), st))
        _lib.check(lib.tk_conv2d_pack_weight(rw.ptr, 1, ctypes.c_void_p(packed.data_ptr()),
                                             ctypes.c_void_p(sums.data_ptr()), st))

        def call():
            arr = arrs[turn[0] % rotate]
            if len(res_refs) > 1:
                a.residual = res_refs[turn[0] % len(res_refs)].ptr
            turn[0] += 1
            _lib.check(lib.tk_qnn_conv2d_block(rx.ptr, ctypes.c_void_p(shadow.data_ptr()), rw.ptr,
                                               ctypes.c_void_p(packed.data_ptr()), ctypes.c_void_p(sums.data_ptr()),
                                               rb.ptr, arr, len(refs), ctypes.byref(a), ctypes.c_void_p(scratch.data_ptr()),
                                               ctypes.c_void_p(sh_out.data_ptr()), st))
        best = [float("inf")] * len(configs)
        for _ in range(reps):
            for ci, cfg in enumerate(configs):
                saved = {k: os.environ.get(k) for k in cfg}
                os.environ.update(cfg)
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    call()
                e1.record()
                e1.synchronize()
                if marker:
                    # a fill kernel between configs: tools/abl_trace.py splits a rocprofv3 kernel
                    # trace at these, so each config's GPU time is read without host overhead
                    torch.empty(1, device=dev).fill_(ci)
                    torch.cuda.synchronize()
                best[ci] = min(best[ci], e0.elapsed_time(e1) / iters * 1e3)
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        out_el = batch * O * OH * OH
        by = x.numel() + w.numel() + 4 * O + out_el * (12 if res else 10)
        macs = out_el * C * K * K
        cols = "  ".join(f"{us:8.1f} us {by / us / 1e3:6.0f} GB/s" for us in best)
        print(f"{name:22s} {cols}   ({2 * macs / best[0] / 1e6:.0f} TOPS)", flush=True)
        tot = [t + u for t, u in zip(tot, best)]
    print("configs:", configs)
    print("sum", "  ".join(f"{t:8.1f} us" for t in tot))


if __name__ == "__main__":
    import json
    cfgs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else None
    main(configs=cfgs, only=sys.argv[2] if len(sys.argv) > 2 else None,
         rotate=int(sys.argv[3]) if len(sys.argv) > 3 else 1, marker="--marker" in sys.argv,
         rotate_res=int(sys.argv[4]) if len(sys.argv) > 4 and not sys.argv[4].startswith("--") else 1)

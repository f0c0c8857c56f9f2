"""Library int8 GEMM reference (torch._int_mm -> hipBLASLt) on the GEMM shapes of ResNet-50's
conv layers at batch 64 (im2col already materialised, so only MFMA + operand streaming)."""
import torch

SHAPES = [("3x3 256->256 14", 64 * 196, 2304, 256), ("3x3 512->512 7", 64 * 49, 4608, 512),
          ("1x1 2048->512 7", 64 * 49, 2048, 512), ("1x1 1024->256 14", 64 * 196, 1024, 256),
          ("3x3 128->128 28", 64 * 784, 1152, 128)]
for name, m, k, n in SHAPES:
    a = torch.randint(-128, 127, (m, k), dtype=torch.int8, device="cuda")
    b = torch.randint(-128, 127, (n, k), dtype=torch.int8, device="cuda").t()
    try:
        for _ in range(3):
            torch._int_mm(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch._int_mm(a, b)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name:20s} M={m} K={k} N={n}: {us:7.1f} us  {2 * m * n * k / us / 1e6:6.0f} TOPS", flush=True)
    except Exception as e:  # noqa: BLE001
        print(name, "int_mm failed:", e, flush=True)

"""Control for the rocprofv3 --memory-copy-trace exit crash: torch alone, no
tachikoma library -- a few 256 MiB device-to-pinned-host copies, then a normal exit.  If this
process also dies inside the profiler's finalisation, the crash belongs to the profiler (ROCm 7.2,
its own libhsa-runtime64) running beside torch's bundled HIP/HSA 7.0 runtime, not to libtachikoma."""
import torch

x = torch.ones(256 << 20, dtype=torch.uint8, device="cuda")
h = torch.empty(x.numel(), dtype=torch.uint8, pin_memory=True)
for _ in range(4):
    h.copy_(x, non_blocking=True)
torch.cuda.synchronize()
print("copies done", int(h[:16].sum()), flush=True)

"""Launch floor on the box: back-to-back tiny kernels (1 workgroup and ~400 workgroups),
event-timed; run under rocprofv3 --kernel-trace for their in-GPU durations."""
import torch

x1 = torch.zeros(64, device="cuda")
x2 = torch.zeros(416 * 256 * 4, device="cuda")
for name, x in (("1 wg", x1), ("416 wg", x2)):
    for _ in range(10):
        x.add_(1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        x.add_(1)
    e1.record()
    e1.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per launch (event-timed)", flush=True)

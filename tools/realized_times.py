"""Per-op-kind device time of a relay.quantize-realized ResNet at the
BASELINE shard size: one compute-only step timed node by node (tk_module_run_profiled), then
traced steps (every record copied to pinned host memory), with algorithmic bytes per kind.
GPU only.

usage: python tools/realized_times.py [depth=50] [batch=64] [reps=3] [qconfig-json]
"""
import json
import sys
import time
from collections import defaultdict

import numpy as np

sys.path.insert(0, ".")
from tachikoma_amd import relay, zoo  # noqa: E402
from tachikoma_amd.contrib import graph_executor  # noqa: E402
from tachikoma_amd.relay.quantize import qconfig, quantize  # noqa: E402


def main(depth=50, batch=64, reps=3, cfg=None):
    depth, batch, reps = int(depth), int(batch), int(reps)
    cfg = json.loads(cfg) if cfg else {}
    m = zoo.resnet_float(depth, batch=batch, hw=224)
    t0 = time.time()
    with qconfig(**cfg):
        q = quantize(m.mod, m.params)
    t_q = time.time() - t0
    lib = relay.build(q, target="mi355x")
    g = graph_executor.GraphModule(lib["default"](0))
    g.set_input("data", m.random_input())
    g.run()
    mod = g.module
    times = np.median(np.array([list(mod.run_profiled().values()) for _ in range(reps)]), axis=0)
    ops = {o.name: o for o in g.plan.ops}
    by = defaultdict(lambda: [0, 0.0, 0])
    for i, (recs, kind) in enumerate(zip(mod.node_records, mod.node_kinds)):
        if not recs:
            by[kind][0] += 1
            by[kind][1] += times[i]
            continue
        head = ops[recs[0]]
        key = head.op if head.op != "ewise" else f"ewise:{head.attrs['ew']}:{head.out.dtype}"
        if head.op in ("nn.conv2d", "nn.dense"):
            key += ":f32"
        nbytes = sum(g.plan.tensor(x).nbytes for x in head.inputs) + sum(ops[r].out.nbytes for r in recs)
        by[key][0] += 1
        by[key][1] += times[i]
        by[key][2] += nbytes
    total = float(times.sum())
    trace_bytes = sum(o.out.nbytes for o in g.plan.ops) + sum(t.nbytes for t in g.plan.inputs)
    # traced steps: every record to pinned host memory
    cap = g.trace_capture()
    import torch
    for _ in range(2):
        g.run(trace=True)
    torch.cuda.synchronize()
    t0 = time.time()
    n_t = 3
    for _ in range(n_t):
        g.run(trace=True)
    cap.synchronize()
    torch.cuda.synchronize()
    traced_ms = (time.time() - t0) / n_t * 1e3
    print(f"realized resnet{depth} batch {batch} qconfig {cfg}: quantize {t_q:.1f} s on the host, "
          f"{len(g.plan.ops)} ops / {mod.n_nodes} nodes, compute-only step {total:.2f} ms "
          f"({batch / total * 1e3:.0f} samples/s), traced step {traced_ms:.1f} ms "
          f"({batch / traced_ms * 1e3:.1f} op-traces/s, {trace_bytes / traced_ms / 1e6:.1f} GB/s of records)")
    print(f"{'op kind':28s} {'nodes':>5s} {'ms':>8s} {'GB/s':>8s}")
    for k, (n, ms, b) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:28s} {n:5d} {ms:8.3f} {b / ms / 1e6 if ms > 0 and b else 0:8.0f}")


if __name__ == "__main__":
    main(*sys.argv[1:])

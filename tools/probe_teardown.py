"""Bisect the rocprofv3 --memory-copy-trace crash at process exit.  The base is what
round-5 stages 0-3 showed exits cleanly under the profiler (r05j, rc 0 each): torch + libtachikoma,
a pinned D2H copy, a LeNet-5 module run untraced, traced host-issued and traced as replayed HIP
graphs with the packed capture, then closed.  Each named feature adds one more piece of what
bench.py does (and bench.py on LeNet-5 does crash, r05i):
  bind    shard.bind_to_gpu_node (sched_setaffinity to the GPU's NUMA node)
  tune    the conv-block find step (tune=True)
  pick    GraphModule.pick_run_mode (host-issued vs graph, timed)
  events  torch timing events around run_range segments on the module's stream
  digest  records_digest + shard.gather_digests (no process group)
  d2h     bench.d2h_probe: 1 GiB pinned D2H copies on one and on two torch streams
  oracle  one sample through oracle/graph_ref's C backend (host threads)
  empty   torch._C._host_emptyCache() after close
  second  a second TraceCapture (bench's file sink double image)
Usage: python tools/probe_teardown.py <stage 0-3> [feature ...]"""
import os
import sys

import torch

sys.path.insert(0, ".")
from tachikoma_amd import _lib, relay, shard, zoo  # noqa: E402
from tachikoma_amd.contrib import graph_executor  # noqa: E402

stage = int(sys.argv[1])
feats = set(sys.argv[2:])
_lib.load()
if "bind" in feats:
    print("placement", shard.bind_to_gpu_node(0), flush=True)
x = torch.ones(1 << 24, dtype=torch.uint8, device="cuda")
h = torch.empty(x.numel(), dtype=torch.uint8, pin_memory=True)
h.copy_(x, non_blocking=True)
torch.cuda.synchronize()
if stage >= 1:
    model = zoo.lenet5(batch=1)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"](0, tune="tune" in feats))
    xin = model.sample_inputs(0, 1)
    m.set_input("data", xin)
    m.run()
    if stage >= 2:
        m.run(trace=True)
        m.trace_capture().synchronize()
    if stage >= 3:
        m.module.use_graph = True
        m.run(trace=True)
        m.trace_capture().synchronize()
    if "second" in feats:
        cap2 = graph_executor.TraceCapture(m.module, m._meta)
        stream = torch.cuda.current_stream()
        cap2.capture_stream.wait_stream(stream)
        cap2.capture_inputs(stream)
        m.module.run(stream, cap2.capture_stream, cap2.host_dst)
        cap2.synchronize()
    if "pick" in feats:
        print("pick", m.pick_run_mode(steps=2), flush=True)
    if "events" in feats:
        stream = torch.cuda.current_stream()
        n = len(m.module.node_kinds)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(3):
            ev[0].record(stream)
            m.module.run_range(0, n // 2, stream)
            m.module.run_range(n // 2, n, stream)
            ev[1].record(stream)
            ev[1].synchronize()
        print("events ms", ev[0].elapsed_time(ev[1]), flush=True)
    if "digest" in feats:
        m.run(trace=True)
        torch.cuda.synchronize()
        print("digests", shard.gather_digests(m.module.records_digest(torch.cuda.current_stream())), flush=True)
    if "oracle" in feats:
        from oracle import graph_ref
        rec = graph_ref.calibrate(model.mod, model.params, {"data": xin[0:1]}, backend="c", threads=4)
        print("oracle records", len(rec), flush=True)
    torch.cuda.synchronize()
    m.close()
    if "second" in feats:
        del cap2
if "d2h" in feats:
    import bench
    print("d2h", bench.d2h_probe(torch.device("cuda", 0)), bench.d2h_probe(torch.device("cuda", 0), streams=2), flush=True)
if "empty" in feats:
    import gc
    gc.collect()
    torch._C._host_emptyCache()
print(f"probe_teardown stage {stage} {sorted(feats)} done", flush=True)

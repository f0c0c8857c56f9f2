"""Bisect the rocprofv3 --memory-copy-trace crash at process exit.  Outcome (round 5):
no feature below reproduces it -- every probe exits 0 -- but each one, like a torch-only process,
sits 30 s in the profiler's finalisation waiting for copy-completion callbacks that never come and
records no copy: the process holds two HSA runtimes (tools/rocprof_one_hsa.sh says why and runs
the profiler with one; bench.py under it exits 0 with its copies traced).
The base is what stages 0-3 showed exits under the profiler (r05j, rc 0 each): torch + libtachikoma,
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
  dist    import torch.distributed first
  order   torch.cuda.current_device() before libtachikoma loads
  chunks  tk_module_set_trace_chunks(8)
  mkev    torch timing events created and never recorded
Usage: python tools/probe_teardown.py <stage 0-3> [feature ...]"""
import os
import sys

import torch

sys.path.insert(0, ".")
from tachikoma_amd import _lib, relay, shard, zoo  # noqa: E402
from tachikoma_amd.contrib import graph_executor  # noqa: E402

stage = int(sys.argv[1])
feats = set(sys.argv[2:])
if "dist" in feats:
    import torch.distributed  # noqa: F401  (bench.py imports it before anything else)
if "order" in feats:
    torch.cuda.current_device()  # bench.py: torch's HIP runtime up before libtachikoma loads
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
    if "chunks" in feats:
        _lib.check(m.module.lib.tk_module_set_trace_chunks(m.module.handle, 8), "tk_module_set_trace_chunks")
    if "mkev" in feats:
        made = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
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
    if "numa" in feats:
        cap = m.trace_capture()
        print("numa pages", shard.numa_pages(cap.ptr, cap.layout.total), flush=True)
    if "meta" in feats:
        from tachikoma_amd.trace_format import read_trace
        m.set_trace_meta(model=model.name, sample_offset=0, rank=0, world=1, n_samples=1)
        m.run(trace=True)
        m.trace_capture().synchronize()
        print("records", len(read_trace(m.trace_capture().bytes()).records), flush=True)
    if "raw" in feats:
        # bench.py's step(): the capture stream waits for the compute stream, timing events on it
        cap = m.trace_capture()
        stream = torch.cuda.current_stream()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for a, z in evs:
            cap.capture_stream.wait_stream(stream)
            a.record(cap.capture_stream)
            cap.capture_inputs(stream)
            m.module.run(stream, cap.capture_stream, cap.host_dst)
            z.record(cap.capture_stream)
        torch.cuda.synchronize()
        print("raw ms", [a.elapsed_time(z) for a, z in evs], flush=True)
    if "compute" in feats:
        for _ in range(3):
            m.run(trace=False)
        torch.cuda.synchronize()
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

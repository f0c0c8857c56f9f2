"""Benchmark: ResNet-50 int8 op-traces/sec on N MI355X (BASELINE.json metric).

A "step" is one traced inference of this rank's batch shard (64 samples of
ResNet-50 int8 224x224 per GPU = BASELINE config 4's per-GPU shard): every op
runs as its own HIP kernel and every op output (plus the graph input) is copied
device→host into the pinned trace image, which after the step holds the complete
tachikoma trace binary of the shard (headers, params, records).  One op-trace =
the complete per-op trace of one sample; value = samples traced by all ranks ÷
max-over-ranks wall time.  Inputs are resident in HBM before timing starts.

Launch: python bench.py [--gpus N --steps K --warmup W]
        (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

INT8_MFMA_PEAK_OPS = 5.0e15  # gfx950 dense int8 (2x the 2.5 PF dense bf16 peak), MI355X_MICROARCH.md
HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (6.3 TB/s measured streaming copy), MI355X_MICROARCH.md


def _log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--model", default="resnet50")
    p.add_argument("--batch", type=int, default=64, help="samples per GPU (shard size)")
    p.add_argument("--cpu-budget-s", type=float, default=15.0, help="CPU baseline time budget")
    p.add_argument("--skip-cpu", action="store_true")
    p.add_argument("--sink", choices=["memory", "file"], default="memory",
                   help="memory: trace image complete in pinned host RAM; file: also write each step to disk")
    p.add_argument("--out-dir", default="/tmp")
    p.add_argument("--no-trace", action="store_true", help="compute-only steps (profiling aid; not the metric)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL over xGMI (one GPU per rank); gloo only to rehearse N>1 on one GPU")
    return p.parse_args()


def cpu_baseline(model_fn, batch_hint: int, budget_s: float):
    """Time the oracle's C restatement (OpenMP port of the reference's int16 conv / int64
    requantize semantics) doing the same per-op record-and-run on the host cores."""
    from oracle import graph_ref
    threads = min(16, len(os.sched_getaffinity(0)))
    model = model_fn(batch=1)
    x_all = model.sample_inputs(0, batch_hint)
    # warm (page in weights, OpenMP pool) on one sample, then as many samples as fit the budget
    t0 = time.perf_counter()
    graph_ref.calibrate(model.mod, model.params, {"data": x_all[:1]}, backend="c", threads=threads)
    one = time.perf_counter() - t0
    n = max(1, min(batch_hint, int(budget_s / max(one, 1e-3))))
    t0 = time.perf_counter()
    for i in range(n):
        graph_ref.calibrate(model.mod, model.params, {"data": x_all[i:i + 1]}, backend="c", threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "op-traces/s", "cores": threads, "kind": "port",
            "sample": f"{n} samples of {model.name} int8 224x224 traced one by one (batch-1 record-and-run, "
                      f"every op output kept), C/OpenMP oracle, {dt:.1f}s"}


def pmc_traffic(model: str, batch: int, launches: int):
    """HBM bytes per launch of the block kernel from the committed PMC summary
    (tools/pmc.sh -> profiles/*_pmc_block.json), when it was taken on this workload."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_block.json")), reverse=True):
        with open(path) as f:
            doc = json.load(f)
        if doc.get("model") == model and doc.get("batch") == batch:
            # per layer-block node (split-K layers dispatch two kernels per node)
            return doc["hbm_bytes_per_step"] / max(launches, 1), os.path.relpath(path, ROOT)
    return None, None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local_rank))
        else:
            torch.cuda.set_device(local_rank % torch.cuda.device_count())
            dist.init_process_group(backend="gloo")
    device = torch.device("cuda", torch.cuda.current_device())
    coll_dev = device if args.dist_backend == "nccl" else torch.device("cpu")

    from tachikoma_amd import relay, shard, zoo
    from tachikoma_amd.contrib import graph_executor

    B = args.batch
    model_fn = zoo.MODELS[args.model]
    model = model_fn(batch=B)
    _log(f"rank {rank}/{world}: building {args.model} batch {B} on {device}")
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"](device.index))
    # weak scaling: B samples per GPU; this rank traces samples [offset, offset + B) of the global batch
    offset, count = shard.shard_range(B * world, world, rank)
    x = model.sample_inputs(offset, count)
    m.set_input("data", x)
    m.set_trace_meta(model=model.name, sample_offset=offset, rank=rank, world=world, n_samples=count)
    cap = m.trace_capture()
    if args.sink == "file":
        os.makedirs(args.out_dir, exist_ok=True)
    _log(f"trace image {cap.layout.total / 1e9:.2f} GB pinned, {len(m.plan.ops)} ops")
    stream = torch.cuda.current_stream(device)

    def barrier():
        if world > 1:
            dist.barrier()

    def step(i):
        if args.no_trace:
            m.run(trace=False)
            torch.cuda.synchronize(device)
            return
        m.run(trace=True)
        cap.synchronize()
        if args.sink == "file":
            cap.write(shard.shard_file(args.out_dir, rank))

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(device)

    # ---- timed region: K traced steps
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(device)
    barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        tc = t.to(coll_dev)
        dist.all_reduce(tc, op=dist.ReduceOp.MAX)
        t = tc
    elapsed_max = float(t.item())

    # ---- compute-only steps (no capture): the kernels alone, each node bracketed by HIP
    # events recorded on the stream the node's kernel runs on (tk_module_set_profiling);
    # the roofline below is taken from these, where no D2H copy shares the device
    torch.cuda.synchronize(device)
    tc = time.perf_counter()
    for _ in range(args.steps):
        m.run(trace=False)
    torch.cuda.synchronize(device)
    compute_ms = (time.perf_counter() - tc) / max(args.steps, 1) * 1e3
    m.module.set_profiling(True)
    node_ms = np.zeros(m.module.n_nodes)
    for _ in range(args.steps):
        m.run(trace=False)
        node_ms += np.array(m.module.node_times())
    m.module.set_profiling(False)
    node_ms /= max(args.steps, 1)

    # ---- roofline of the dominant kernel: the fused MFMA conv/dense layer block
    # (qnn.conv2d|dense -> bias_add -> requantize [-> qnn.add(residual)] [-> clip] in one
    # kernel).  It is bound by HBM: every op output of the block is a trace record that must
    # be written (int32 conv + int32 bias_add + int8 requantize [+ int8 add] + int8 clip per
    # output element); algorithmic bytes = input + weights + bias [+ residual] + records.
    blk_ops, blk_bytes, blk_ms, n_launch = 0.0, 0.0, 0.0, 0
    ops_by_name = {o.name: o for o in m.plan.ops}
    for i, recs in enumerate(m.module.node_records):
        if not recs or m.module.node_kinds[i] not in ("conv_block", "dense_block", "qnn.conv2d", "qnn.dense"):
            continue
        op = ops_by_name[recs[0]]
        x = m.plan.tensor(op.inputs[0])
        w = m.plan.tensor(op.inputs[1])
        out_elems = int(np.prod(op.out.shape))
        if op.op == "qnn.conv2d":
            o, cg, kh, kw = w.shape
            nb, _, oh, ow = op.out.shape
            macs = nb * o * oh * ow * cg * kh * kw
        else:
            macs = op.out.shape[0] * w.shape[0] * w.shape[1]
        rec_bytes = sum(ops_by_name[r].out.nbytes for r in recs)
        # a fused residual join also reads the other qnn.add operand
        res_bytes = sum(ops_by_name[r].out.nbytes for r in recs if ops_by_name[r].op == "qnn.add")
        blk_bytes += x.nbytes + w.nbytes + (4 * op.out.shape[1] if len(recs) > 1 else 0) + rec_bytes + res_bytes
        blk_ops += 2.0 * macs
        blk_ms += node_ms[i]
        n_launch += 1
    achieved_bw = blk_bytes / (blk_ms * 1e-3) if blk_ms > 0 else 0.0
    achieved_ops = blk_ops / (blk_ms * 1e-3) if blk_ms > 0 else 0.0
    total_ms = float(node_ms.sum())
    traffic, traffic_src = pmc_traffic(args.model, B, n_launch)

    # ---- trace-digest all-gather (RCCL over xGMI): one u64 record digest per rank, computed
    # on the device over the records of the last traced step (outside the timed region)
    m.run(trace=not args.no_trace)
    if not args.no_trace:
        cap.synchronize()
    digests = shard.gather_digests(m.module.records_digest(stream).to(coll_dev))
    if args.sink == "file" and not args.no_trace:
        path = shard.shard_file(args.out_dir, rank)
        cap.write(path)
        entries = [shard.ShardEntry(r, *shard.shard_range(B * world, world, r), shard.hex64(d),
                                    shard.shard_file(args.out_dir, r)) for r, d in enumerate(digests)]
        if rank == 0:
            shard.write_manifest(os.path.join(args.out_dir, "trace.manifest.json"), model.name, B * world, entries)

    if rank == 0:
        traces = B * world * args.steps
        value = traces / elapsed_max
        cpu = None
        if not args.skip_cpu and world == 1:  # reported on rank 0 at N = 1 only
            _log("cpu baseline (oracle port) ...")
            cpu = cpu_baseline(model_fn, B, args.cpu_budget_s)
        macs_per_sample = zoo.macs_per_sample(model_fn(batch=1))
        trace_bytes = cap.layout.total
        line = {
            "metric": "ResNet-50 int8 op-traces/sec at 1/2/4/8 GPU; bit-exact vs CPU",
            "value": round(value, 3),
            "unit": "op-traces/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": "synthetic (seeded int8 inputs, random-init int8 weights of the ResNet-50 v1 topology)",
            "config": {"workload": f"{args.model} int8 224x224, {B} samples per GPU (BASELINE config 4 shard), "
                                   f"full per-op trace to pinned host memory",
                       "model": args.model, "global_batch": B * world, "samples_per_gpu": B, "seq_len": None,
                       "parallelism": f"batch-shard x{world}", "sink": args.sink},
            "roofline": {"bound": "hbm", "achieved": round(achieved_bw / 1e9, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved_bw / 1e9 / HBM_PEAK_GBPS, 4),
                         "traffic": None if traffic is None else int(traffic),
                         "traffic_unit": "HBM bytes per layer-block node (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, per step / nodes)",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_node": int(blk_bytes / max(n_launch, 1)),
                         "kernel": "gemm_i8_kernel<*,*,block> fused conv/dense layer block (v_mfma_i32_32x32x32_i8)",
                         "nodes_per_step": n_launch, "kernel_ms_per_step": round(blk_ms, 3),
                         "algorithmic_bytes_per_step": int(blk_bytes),
                         "mfma_tops": round(achieved_ops / 1e12, 1),
                         "mfma_frac": round(achieved_ops / INT8_MFMA_PEAK_OPS, 4)},
            "cpu_baseline": cpu,
            "extra": {
                "compute_only_ms_per_step": round(compute_ms, 3),
                "compute_only_traces_per_s": round(B * world / (compute_ms * 1e-3), 1),
                "all_node_ms_per_step": round(total_ms, 3),
                "trace_bytes_per_step": trace_bytes,
                "trace_GBps_per_gpu": round(trace_bytes / (elapsed_max / args.steps) / 1e9, 2),
                "macs_per_sample": macs_per_sample,
                "ops_per_sample": 2 * macs_per_sample,
                "record_digests": [shard.hex64(d) for d in digests],
            },
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

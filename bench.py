"""Benchmark: ResNet-50 int8 op-traces/sec on N MI355X (BASELINE.json metric).

A "step" is one traced inference of this rank's batch shard (64 samples of
ResNet-50 int8 224x224 per GPU = BASELINE config 4's per-GPU shard): every op
runs as its own HIP kernel and every op output (plus the graph input) is copied
device→host into the pinned trace image, which after the step holds the complete
tachikoma trace binary of the shard (headers, params, records).  One op-trace =
the complete per-op trace of one sample; value = samples traced by all ranks ÷
max-over-ranks wall time.  Inputs are resident in HBM before timing starts.

Launch: python bench.py [--gpus N --steps K --warmup W]
  * N > 1 without torch.distributed.run: this process starts N rank processes (before any
    GPU call) and exits with their status; with torch.distributed.run (WORLD_SIZE set),
    WORLD_SIZE must equal --gpus.
  * --dist-backend gloo rehearses N ranks on one GPU (all ranks share cuda:0).

After the timed region, the trace image is checked record for record against the CPU
oracle: at N > 1 every rank checks ceil(64 / N) samples spread over its shard, and rank 0 then
times the CPU baseline at every N, checking each sample it traces and then (untimed) the rest of
its shard -- at N = 1 all 64 samples; any mismatch makes the run exit non-zero.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

INT8_MFMA_PEAK_OPS = 5.0e15  # gfx950 dense int8 (2x the 2.5 PF dense bf16 peak), MI355X_MICROARCH.md
HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (6.3 TB/s measured streaming copy), MI355X_MICROARCH.md
MFMA_SIMDS = 1024            # 256 CUs x 4 SIMDs
PEAK_CLOCK_HZ = 2.4e9        # MI355X peak engine clock (5.0 POPS int8 = 1024 SIMDs x 2048 ops/cycle x 2.4 GHz)
METRIC = "ResNet-50 int8 op-traces/sec at 1/2/4/8 GPU; bit-exact vs CPU"
# the BASELINE.json config each --model measures (configs 3 and 5 are single-GPU batch-64 workloads)
WORKLOADS = {
    "resnet50": ("BASELINE config 4 shard", "ResNet-50 v1"),
    "resnet18": ("BASELINE config 3", "ResNet-18 (torchvision v1)"),
    "mobilenet_v2": ("BASELINE config 5", "MobileNetV2 1.0"),
}


def metric_for(model: str) -> str:
    """BASELINE.json's metric for the headline model; the same unit named for configs 3 and 5."""
    if model == "resnet50":
        return METRIC
    return f"{WORKLOADS.get(model, ('', model))[1]} int8 op-traces/sec; bit-exact vs CPU"
BLOCK_KINDS = ("conv_block", "dense_block", "qnn.conv2d", "qnn.dense")


def _log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--model", default="resnet50")
    p.add_argument("--batch", type=int, default=64, help="samples per GPU (shard size)")
    p.add_argument("--cpu-budget-s", type=float, default=15.0, help="CPU baseline time budget")
    p.add_argument("--skip-cpu", action="store_true")
    p.add_argument("--sink", choices=["memory", "file"], default="memory",
                   help="memory: trace image complete in pinned host RAM; file: also write every step's image "
                        "to trace.rank<r>.tkt, overlapped with the next step (two pinned images, writer thread)")
    p.add_argument("--out-dir", default="/tmp")
    p.add_argument("--file-overlap", choices=["on", "off", "auto"], default="auto",
                   help="file sink: write image i while step i+1 runs (on), finish each write before the next "
                        "step starts (off: no D2H / writer concurrency), or auto: time 3 steps of each before the "
                        "warm-up and keep the faster (the writer and the next step's D2H slow each other by "
                        "box-dependent amounts: overlapped won on one round-4 box, 126.8 vs 107.7 op-traces/s, and "
                        "lost on another, 89.3 vs 106.2)")
    p.add_argument("--no-trace", action="store_true", help="compute-only steps (profiling aid; not the metric)")
    p.add_argument("--tune-report", default=None, help="write the find step's per-node kernel timings (JSON) here")
    p.add_argument("--tune-table", default="auto",
                   help="conv-block kernels: 'auto' replays the committed find-step table for this workload "
                        "(profiles/*_tune_table.json, newest) so that the timed run uses the kernels the committed "
                        "profiles were taken on, falling back to the find step when none applies; a path replays "
                        "that table; 'none' runs the find step on this GPU")
    p.add_argument("--write-tune-table", default=None, help="write the kernel choice this run used as a tune table")
    p.add_argument("--run-mode", choices=["graph", "host", "auto"], default="graph",
                   help="traced-step submission: one replayed HIP graph per step (tk_module_run_graph, the "
                        "default: immune to a host that issues calls late, profiles/r03r_run_modes_slow_host.txt), "
                        "every kernel and copy issued from the host (tk_module_run), or auto = the faster of the "
                        "two over two steps before the warm-up (GraphModule.pick_run_mode)")
    p.add_argument("--graph-copies", type=int, default=0,
                   help="graph runs' record copies (tk_module_set_graph_copies): 0 packed image chunks copied by "
                        "host-issued SDMA copies (default), 1 copy kernels, 2-4 memcpy nodes in that many chains, "
                        "5 one chain")
    p.add_argument("--trace-chunks", type=int, default=8, help="chunks of the packed capture (tk_module_set_trace_chunks)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL over xGMI (one GPU per rank); gloo only to rehearse N>1 on one GPU")
    p.add_argument("--no-numa-bind", action="store_true", help="do not bind ranks to their GPU's NUMA node")
    p.add_argument("--copy-trace", default=None,
                   help="after the timed region, trace 3 more packed steps with per-chunk copy timing "
                        "(tk_module_copy_trace: the in-process memory-copy trace of the real step) into this JSON file")
    p.add_argument("--force-pg", action="store_true",
                   help="start the process group and run the N>1 collectives (elapsed all-reduce, record-digest "
                        "all-gather, rank-info all-gather, status broadcast) even at one rank: exercises the RCCL "
                        "branch on a single GPU")
    return p.parse_args(argv)


# ---------------------------------------------------------------- N-rank launcher

def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, cmd) -> int:
    """`python bench.py --gpus N`: one process per GPU running `cmd`, started before this
    process touches the GPU (the parent never initialises HIP); rank r gets RANK = LOCAL_RANK
    = r and a torch.distributed rendezvous on 127.0.0.1.  Rank 0 prints the JSON line; the
    exit status is the first non-zero rank status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(list(cmd), env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            time.sleep(0.2)
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code and not rc:
                    rc = code
                    for q in live:  # one rank failed: the others would block in a collective
                        q.terminate()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


# ---------------------------------------------------------------- host facts

def cpu_quota() -> float | None:
    """CPUs granted by the cgroup (cpu.max quota / period), None when unlimited/unknown."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()
            if q != "max":
                return int(q) / int(per)
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def d2h_probe(device, nbytes: int = 1 << 30, reps: int = 4, streams: int = 1) -> float:
    """Pinned device→host bandwidth (GB/s) of `nbytes` moved by `streams` concurrent
    hipMemcpyAsync copies (nbytes / streams each, one side stream per copy), timed with HIP
    events from a common start: the PCIe ceiling the traced steps are compared with."""
    import torch
    src = torch.empty(nbytes, dtype=torch.uint8, device=device)
    src.fill_(1)
    dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    ss = [torch.cuda.Stream(device=device) for _ in range(streams)]
    part = nbytes // streams
    best = 0.0
    for r in range(reps + 1):  # the first repetition warms page tables and the SDMA queues
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(ss[0])
        for k, s in enumerate(ss):
            s.wait_event(e0)
            with torch.cuda.stream(s):
                dst[k * part:(k + 1) * part].copy_(src[k * part:(k + 1) * part], non_blocking=True)
        for s in ss[1:]:
            ss[0].wait_stream(s)
        e1.record(ss[0])
        e1.synchronize()
        if r:
            best = max(best, part * streams / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del src, dst
    return best


# ---------------------------------------------------------------- CPU baseline + parity

class Parity:
    """Record-by-record comparison of the GPU trace image with the CPU oracle's records."""

    def __init__(self, records):
        self.records = records          # {name: [B_shard, ...]} views into the trace image
        self.samples = 0
        self.n_records = 0
        self.mismatches = 0
        self.first = None
        self.seen = set()

    def check(self, local_index: int, global_index: int, expected) -> None:
        """A sample checked twice (parity spread, then the CPU baseline) is compared again but
        counted once."""
        fresh = local_index not in self.seen
        self.seen.add(local_index)
        self.samples += fresh
        for name, exp in expected.items():
            self.n_records += fresh
            got = self.records[name][local_index:local_index + 1]
            if got.shape != exp.shape or got.dtype != exp.dtype or not np.array_equal(got, exp):
                self.mismatches += 1
                if self.first is None:
                    where = None
                    if got.shape == exp.shape:
                        bad = np.argwhere(got != exp)[0]
                        where = {"index": [int(v) for v in bad[1:]], "gpu": int(got[tuple(bad)]),
                                 "cpu": int(exp[tuple(bad)])}
                    self.first = {"sample": global_index, "record": name, **(where or {"shape": list(got.shape)})}

    def summary(self) -> dict:
        return {"samples": self.samples, "records": self.n_records, "mismatches": self.mismatches,
                "first_mismatch": self.first}


def spread_samples(count: int, n: int):
    """n local sample indices spread evenly over a shard of `count` (first and last included)."""
    n = max(1, min(count, n))
    return sorted(set(int(round(v)) for v in np.linspace(0, count - 1, n)))


def cpu_baseline(model_fn, offset: int, batch: int, budget_s: float, threads: int, parity: Parity):
    """Time the oracle's C restatement (OpenMP port of the reference's int16 conv / int64
    requantize semantics) doing the same per-op record-and-run, one sample at a time, on
    `threads` host cores; every sample it traces is also checked against the GPU trace, and so are
    the shard's other samples (untimed), so that the in-run parity covers the whole shard."""
    from oracle import graph_ref
    model = model_fn(batch=1)
    one = model.sample_inputs(offset, 1)
    t0 = time.perf_counter()
    rec = graph_ref.calibrate(model.mod, model.params, {"data": one}, backend="c", threads=threads)
    first = time.perf_counter() - t0  # includes paging in the weights / OpenMP pool start
    parity.check(0, offset, rec)
    del rec
    n = max(1, min(batch - 1, int(budget_s / max(first, 1e-3))))
    picks = sorted(set(int(round(v)) for v in np.linspace(1, batch - 1, n))) if batch > 1 else []
    dt = 0.0
    for i in picks:
        x = model.sample_inputs(offset + i, 1)
        t0 = time.perf_counter()
        rec = graph_ref.calibrate(model.mod, model.params, {"data": x}, backend="c", threads=threads)
        dt += time.perf_counter() - t0
        parity.check(i, offset + i, rec)
        del rec
    timed = len(picks) or 1
    if not picks:
        dt = first
    # the shard's other samples are checked too (untimed): in-run parity covers the whole shard
    for i in sorted(set(range(1, batch)) - set(picks)):
        rec = graph_ref.calibrate(model.mod, model.params, {"data": model.sample_inputs(offset + i, 1)}, backend="c",
                                  threads=threads)
        parity.check(i, offset + i, rec)
        del rec
    return {"value": round(timed / dt, 3), "unit": "op-traces/s", "cores": threads, "kind": "port",
            "sample": f"{timed} samples of {model.name} int8 224x224 spread over the shard, traced one by one "
                      f"(batch-1 record-and-run, every op output kept), C/OpenMP oracle on {threads} threads, "
                      f"{dt:.1f}s timed (first sample excluded as warm-up)"}


def pmc_traffic(model: str, batch: int, library: str, tune_digest: str | None = None):
    """HBM traffic of the block kernel from a committed PMC summary (tools/pmc.sh ->
    profiles/*_pmc_block.json) taken on this workload: preferably the one taken with this run's
    kernel mix (the same tune table, by digest) and library; failing that the newest by its
    embedded UTC stamp (never by file name).  Returns per launch / per step bytes, launches per
    step, the source and whether library and kernel mix match."""
    import glob
    docs = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "*_pmc_block.json")):
        with open(path) as f:
            doc = json.load(f)
        if doc.get("model") == model and doc.get("batch") == batch and doc.get("created_utc"):
            kern = tune_digest is not None and doc.get("tune_table_digest") == tune_digest
            docs.append((kern, doc.get("library") == library, doc["created_utc"], path, doc))
    if not docs:
        return None
    kern, same, _, path, doc = max(docs, key=lambda d: (d[0], d[1], d[2]))
    launches = int(doc["launches_per_step"])  # dispatches: a split-K node launches twice
    return {"per_launch": doc["hbm_bytes_per_step"] / max(launches, 1), "per_step": doc["hbm_bytes_per_step"],
            "launches": launches, "source": os.path.relpath(path, ROOT), "library_match": same,
            "kernel_match": kern, "library": doc.get("library"), "mfma": doc.get("mfma")}


def find_tune_table(model: str, batch: int):
    """The newest committed find-step table for this workload (profiles/*_tune_table.json, by its
    embedded UTC stamp), or None."""
    import glob
    best = None
    for path in glob.glob(os.path.join(ROOT, "profiles", "*_tune_table.json")):
        with open(path) as f:
            doc = json.load(f)
        if doc.get("model") == model and doc.get("batch") == batch and doc.get("created_utc"):
            if best is None or doc["created_utc"] > best[0]:
                best = (doc["created_utc"], path)
    return None if best is None else best[1]


# ---------------------------------------------------------------- one rank

def dump_maps_at_exit() -> None:
    """TK_DUMP_MAPS=path: write /proc/self/maps there (the mapping the process exits with), so that
    raw PCs of a crash during exit (glog / rocprofv3 backtraces) can be symbolised offline."""
    path = os.environ.get("TK_DUMP_MAPS")
    if path:
        with open("/proc/self/maps") as src, open(path, "w") as dst:
            dst.write(src.read())

def check_gpu_count(args) -> None:
    """`--gpus N` over RCCL needs N visible GPUs (one rank per GPU): fail at once, before any rank
    starts or ``init_process_group("nccl")`` waits on a rank that cannot exist.  Counting devices
    does not initialise HIP.  The gloo backend rehearses N ranks on fewer GPUs and is exempt."""
    if args.dist_backend != "nccl" or args.gpus <= 1:
        return
    import torch
    have = torch.cuda.device_count()
    if args.gpus > have:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs (one rank per GPU over "
                         f"RCCL), this host shows {have}; use --dist-backend gloo to rehearse N ranks on one GPU")


def pick_overlap(rounds: dict) -> dict:
    """The file sink's overlap pick from interleaved rounds of ms per step, {"on": [...], "off":
    [...]}: each mode's median over the rounds after the first (the disk settles during the first
    round), the faster mode picked (ties go to "on")."""
    med = {k: round(float(np.median(v[1:] if len(v) > 1 else v)), 1) for k, v in rounds.items()}
    return dict(med, pick=min(("on", "off"), key=lambda k: med[k]),
                rounds_ms={k: [round(x, 1) for x in v] for k, v in rounds.items()})


def host_id() -> str:
    """The physical host: its kernel's boot id (containers on one host share it; the hostname is
    the container's).  Tells two boxes' runs apart in the line."""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            return f.read().strip()
    except OSError:
        return os.uname().nodename


def mount_of(path: str):
    """(mount point, filesystem type, device) of the mount holding `path` (/proc/mounts)."""
    best = None
    real = os.path.realpath(path)
    try:
        with open("/proc/mounts") as f:
            for line in f:
                dev, mnt, fstype = line.split()[:3]
                if (real == mnt or real.startswith(mnt.rstrip("/") + "/")) and (best is None or len(mnt) > len(best[0])):
                    best = (mnt, fstype, dev)
    except OSError:
        return None
    return None if best is None else {"mount": best[0], "type": best[1], "device": best[2]}


def main(argv=None) -> int:
    args = parse(argv)
    check_gpu_count(args)
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        return launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] +
                            (sys.argv[1:] if argv is None else list(argv)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    home_cpus = os.sched_getaffinity(0)

    import torch
    import torch.distributed as dist

    pg = world > 1 or args.force_pg  # the collectives below run whenever a process group exists
    if pg and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if pg:
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local_rank))
        else:
            torch.cuda.set_device(local_rank % torch.cuda.device_count())
            dist.init_process_group(backend="gloo")
    device = torch.device("cuda", torch.cuda.current_device())
    coll_dev = device if args.dist_backend == "nccl" else torch.device("cpu")

    from tachikoma_amd import _lib, relay, shard, zoo
    from tachikoma_amd.contrib import graph_executor
    from tachikoma_amd.trace_format import read_trace

    # NUMA: this rank's CPUs (and so its pinned trace image) on its GPU's socket
    placement = {"pci": None, "numa_node": None, "cpus": len(home_cpus), "bound": False}
    if not args.no_numa_bind:
        placement = shard.bind_to_gpu_node(device.index)

    B = args.batch
    model_fn = zoo.MODELS[args.model]
    model = model_fn(batch=B)
    _log(f"rank {rank}/{world}: building {args.model} batch {B} on {device} "
         f"(numa node {placement['numa_node']}, {placement['cpus']} cpus)")
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    # conv-block kernels: a committed / given tune table (the kernels the committed profiles were
    # taken on) or the find step on this GPU (tk_module_tune)
    table = None if args.tune_table == "none" else (find_tune_table(args.model, B) if args.tune_table == "auto"
                                                    else args.tune_table)
    tune_info = {"source": "find step on this GPU", "table": None}
    try:
        m = graph_executor.GraphModule(lib["default"](device.index, tune=table or True))
        if table:
            tune_info = {"source": "tune table", "table": os.path.relpath(table, ROOT)}
    except _lib.TachikomaError as e:
        if args.tune_table != "auto":
            raise
        _log(f"tune table {table} does not apply ({e}); running the find step")
        m = graph_executor.GraphModule(lib["default"](device.index))
        tune_info = {"source": "find step on this GPU (table did not apply)", "table": None}
    tune_info["digest"] = m.module.tune_table_digest
    m.module.use_graph = args.run_mode == "graph"
    if args.graph_copies:
        _lib.check(m.module.lib.tk_module_set_graph_copies(m.module.handle, args.graph_copies),
                   "tk_module_set_graph_copies")
    _lib.check(m.module.lib.tk_module_set_trace_chunks(m.module.handle, args.trace_chunks), "tk_module_set_trace_chunks")
    tuning = m.module.tuning
    if args.tune_report and rank == 0:
        with open(args.tune_report, "w") as f:
            json.dump(tuning, f, indent=1)
    if args.write_tune_table and rank == 0:
        doc = m.module.tuning_table()
        doc.update(model=args.model, batch=B, created_utc=time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
        with open(args.write_tune_table, "w") as f:
            json.dump(doc, f, indent=1)
    # weak scaling: B samples per GPU; this rank traces samples [offset, offset + B) of the global batch
    offset, count = shard.shard_range(B * world, world, rank)
    x = model.sample_inputs(offset, count)
    m.set_input("data", x)
    m.set_trace_meta(model=model.name, sample_offset=offset, rank=rank, world=world, n_samples=count)
    caps = [m.trace_capture()]
    if args.sink == "file" and not args.no_trace:
        caps.append(graph_executor.TraceCapture(m.module, m._meta))  # second image: write i while i+1 runs
        os.makedirs(args.out_dir, exist_ok=True)
    image_pages = shard.numa_pages(caps[0].ptr, caps[0].layout.total)
    _log(f"trace image {caps[0].layout.total / 1e9:.2f} GB pinned x{len(caps)} "
         f"(pages per node {image_pages}), {len(m.plan.ops)} ops")
    stream = torch.cuda.current_stream(device)
    path = shard.shard_file(args.out_dir, rank)

    def teardown():
        # while the HIP runtime is alive: device idle, native module destroyed, pinned images
        # released -- nothing is left for finalisers or library static destructors at exit
        caps.clear()
        m.close()
        import gc
        gc.collect()
        torch._C._host_emptyCache()  # the pinned trace images go back to the driver now, not at exit
        dump_maps_at_exit()

    # TK_BENCH_STOP=<phase>: end the run (same teardown) right after that phase -- bisects what in
    # this process a profiler's exit trips over
    stop_at = os.environ.get("TK_BENCH_STOP")

    def stop(phase):
        if stop_at == phase:
            _log(f"TK_BENCH_STOP: ending after {phase}")
            teardown()
            return True
        return False

    if stop("setup"):
        return 0

    import concurrent.futures
    writer = concurrent.futures.ThreadPoolExecutor(max_workers=1) if len(caps) > 1 else None
    pending = [None] * len(caps)

    def write_image(cap):
        cap.synchronize()
        cap.write(path)

    # per-step D2H telemetry: HIP events on the capture stream bracket each timed step's copies
    # (graph input + every record), so a slow host link shows in the line itself
    rec_bytes = sum(int(np.prod(t.shape, dtype=np.int64)) * np.dtype(t.dtype).itemsize for t in m.plan.records)
    d2h_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]

    overlap_mode = ["off" if args.file_overlap == "off" else "on"]

    def step(i, timed=False):
        if args.no_trace:
            m.run(trace=False)
            return
        k = i % len(caps)
        cap = caps[k]
        if writer is not None and pending[k] is not None:
            pending[k].result()  # the writer is done with this image: it may be overwritten
        # memory sink: the next run's kernels wait for this run's copies on the device
        # (tk_module_run's capture event), the host does not block between steps
        cap.capture_stream.wait_stream(stream)
        if timed:
            d2h_ev[i][0].record(cap.capture_stream)
        cap.capture_inputs(stream)
        m.module.run(stream, cap.capture_stream, cap.host_dst)
        if timed:
            d2h_ev[i][1].record(cap.capture_stream)
        if writer is not None:
            pending[k] = writer.submit(write_image, cap)
            if overlap_mode[0] == "off":
                pending[k].result()

    def drain():
        for k, f in enumerate(pending):
            if f is not None:
                f.result()
                pending[k] = None
        torch.cuda.synchronize(device)  # every stream, the capture streams included

    def barrier():
        if pg:
            dist.barrier()

    # submission find step (untimed): host-issued vs one replayed HIP graph per traced step
    mode_pick = None
    if args.run_mode == "auto" and not args.no_trace:
        mode_pick = m.pick_run_mode(steps=2)
        torch.cuda.synchronize(device)
    overlap_pick = None
    if writer is not None and args.file_overlap == "auto":
        # the sink's find step (untimed): overlapped vs serialised, 3 steps each, interleaved over
        # 5 rounds (on, off, on, off, ...) so that a box's disk drifting between probes (10.5-16.7
        # GB/s on one round-4 box) hits both modes alike; each mode's median over rounds 2-5 is
        # compared (the first rounds run slow while the disk settles: r05r's on / off rounds were
        # 860 / 985, 817 / 608, 555 / 606 ms per step, and a median over all three picked "off",
        # frac 0.77, where the overlapped run reached 0.90)
        rounds = {"on": [], "off": []}
        for _ in range(5):
            for mode in ("on", "off"):
                overlap_mode[0] = mode
                step(0)
                drain()
                tp = time.perf_counter()
                for i in range(3):
                    step(i)
                drain()
                rounds[mode].append((time.perf_counter() - tp) / 3 * 1e3)
        overlap_pick = pick_overlap(rounds)
        overlap_mode[0] = overlap_pick["pick"]
    if stop("pick"):
        return 0
    for i in range(args.warmup):
        step(i)
    drain()
    # file sink: the same writer alone on the same filesystem before the timed region too (the
    # disk's solo rate varies between probes on one box, 10.5-16.7 GB/s in round 4): the sink's
    # ceiling is the best of the probes before and after
    probe_s = []
    if args.sink == "file" and not args.no_trace:
        probe_path = path + ".probe"
        for _ in range(2):
            tp = time.perf_counter()
            caps[0].write(probe_path)
            probe_s.append(time.perf_counter() - tp)
        os.remove(probe_path)

    # ---- timed region: K traced steps
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, timed=True)
    drain()
    barrier()
    elapsed = time.perf_counter() - t0
    step_gbps = [] if args.no_trace else \
        [rec_bytes / (a.elapsed_time(z) * 1e-3) / 1e9 for a, z in d2h_ev]
    if stop("timed"):
        return 0

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if pg:
        tc = t.to(coll_dev)
        dist.all_reduce(tc, op=dist.ReduceOp.MAX)
        t = tc
    elapsed_max = float(t.item())
    if writer is not None:
        writer.shutdown()

    # ---- copy trace of the real traced step (packed graph mode): per chunk, bytes and the copy's
    # start / end on the capture stream after the step's first launch; gaps between chunk copies
    # are time the PCIe link idles inside a step
    copy_trace = None
    if args.copy_trace and not args.no_trace and m.module.use_graph and args.graph_copies == 0:
        m.module.set_copy_trace(True)
        steps_ct = []
        for i in range(3):
            step(i)
            drain()
            ch = m.module.copy_trace()
            busy = sum(c["end_ms"] - c["start_ms"] for c in ch)
            gaps = [round(b["start_ms"] - a["end_ms"], 4) for a, b in zip(ch, ch[1:])]
            tot = sum(c["bytes"] for c in ch)
            steps_ct.append({"chunks": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in c.items()} for c in ch],
                             "bytes": tot, "copy_busy_ms": round(busy, 3),
                             "first_copy_start_ms": round(ch[0]["start_ms"], 3) if ch else None,
                             "last_copy_end_ms": round(ch[-1]["end_ms"], 3) if ch else None,
                             "gaps_ms": gaps, "GBps_while_copying": round(tot / (busy * 1e-3) / 1e9, 2) if busy else None,
                             "GBps_first_to_last": round(tot / ((ch[-1]["end_ms"] - ch[0]["start_ms"]) * 1e-3) / 1e9, 2)
                             if ch else None})
        m.module.set_copy_trace(False)
        copy_trace = {"source": "tk_module_copy_trace (HIP timing events around each chunk copy on the capture stream)",
                      "steps": steps_ct}
        if rank == 0:
            with open(args.copy_trace, "w") as f:
                json.dump(copy_trace, f, indent=1)

    # ---- compute-only steps (no capture): the kernels alone, timed with HIP events recorded
    # on the stream they run on (torch's current stream, handed to the module); the roofline
    # below is taken from these, where no D2H copy shares the device
    torch.cuda.synchronize(device)
    tc0 = time.perf_counter()
    for _ in range(args.steps):
        m.run(trace=False)
    torch.cuda.synchronize(device)
    compute_ms = (time.perf_counter() - tc0) / max(args.steps, 1) * 1e3
    if stop("compute"):
        return 0
    # Block time from HIP events bracketing each maximal run of consecutive block nodes (52 of
    # ResNet-50's 54 blocks are one run): a timing event between every two nodes would add the
    # command processor's ~5.6 us per event to every node (rocprof: kernels back to back have
    # no gap, event-separated ones 5.4-5.9 us, profiles/r02d_network_kernels.txt).
    kinds = m.module.node_kinds
    is_blk = [bool(recs) and kinds[i] in BLOCK_KINDS for i, recs in enumerate(m.module.node_records)]
    segs = []
    for i, f in enumerate(is_blk):
        if segs and segs[-1][2] == f:
            segs[-1][1] = i + 1
        else:
            segs.append([i, i + 1, f])
    blk_segs = [sg for sg in segs if sg[2]]
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in blk_segs]
    step_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    blk_ms, step_ms = 0.0, 0.0
    for _ in range(args.steps):
        step_ev[0].record(stream)
        k = 0
        for b, e, f in segs:
            if f:
                evs[k][0].record(stream)
                m.module.run_range(b, e, stream)
                evs[k][1].record(stream)
                k += 1
            else:
                m.module.run_range(b, e, stream)
        step_ev[1].record(stream)
        step_ev[1].synchronize()
        blk_ms += sum(a.elapsed_time(z) for a, z in evs)
        step_ms += step_ev[0].elapsed_time(step_ev[1])
    blk_ms /= max(args.steps, 1)
    step_ms /= max(args.steps, 1)
    if stop("blocks"):
        return 0

    # ---- roofline of the dominant kernel: the fused MFMA conv/dense layer block
    # (qnn.conv2d|dense -> bias_add -> requantize [-> qnn.add(residual)] [-> clip] in one
    # kernel).  It is bound by HBM: every op output of the block is a trace record that must
    # be written (int32 conv + int32 bias_add + int8 requantize [+ int8 add] + int8 clip per
    # output element); algorithmic bytes = input + weights + bias [+ residual] + records.
    blk_ops, blk_bytes, n_launch = 0.0, 0.0, 0
    ops_by_name = {o.name: o for o in m.plan.ops}
    for i, recs in enumerate(m.module.node_records):
        if not is_blk[i]:
            continue
        op = ops_by_name[recs[0]]
        xin = m.plan.tensor(op.inputs[0])
        w = m.plan.tensor(op.inputs[1])
        if op.op == "qnn.conv2d":
            o, cg, kh, kw = w.shape
            nb, _, oh, ow = op.out.shape
            macs = nb * o * oh * ow * cg * kh * kw
        else:
            macs = op.out.shape[0] * w.shape[0] * w.shape[1]
        rec_bytes = sum(ops_by_name[r].out.nbytes for r in recs)
        # a fused residual join also reads the other qnn.add operand
        res_bytes = sum(ops_by_name[r].out.nbytes for r in recs if ops_by_name[r].op == "qnn.add")
        blk_bytes += xin.nbytes + w.nbytes + (4 * op.out.shape[1] if len(recs) > 1 else 0) + rec_bytes + res_bytes
        blk_ops += 2.0 * macs
        n_launch += 1
    achieved_bw = blk_bytes / (blk_ms * 1e-3) if blk_ms > 0 else 0.0
    achieved_ops = blk_ops / (blk_ms * 1e-3) if blk_ms > 0 else 0.0
    total_ms = step_ms
    pmc = pmc_traffic(args.model, B, _lib.build_info(), m.module.tune_table_digest)

    # ---- trace-digest all-gather (RCCL over xGMI): one u64 record digest per rank, computed
    # on the device over the records of one more traced step (outside the timed region); the
    # image it leaves is the one checked below
    m.run(trace=not args.no_trace)
    torch.cuda.synchronize(device)
    digests = shard.gather_digests(m.module.records_digest(stream).to(coll_dev))
    if stop("digest"):
        return 0
    file_check = None
    if args.sink == "file" and not args.no_trace:
        caps[0].write(path)
        # the file on disk must carry exactly the records the device digested
        from tachikoma_amd.trace_format import trace_file_digest
        fd = trace_file_digest(path)
        file_check = {"path": path, "filesystem": mount_of(path), "overlap": overlap_mode[0],
                      "overlap_pick_ms_per_step": overlap_pick,
                      "writer": {k: os.environ[k] for k in ("TK_WRITE_THREADS", "TK_WRITE_PIECE_MB", "TK_WRITE_BUFFERED")
                                 if os.environ.get(k)} or "default (O_DIRECT, 256 MiB pieces, 2 threads)",
                      "file_digest": shard.hex64(fd), "device_digest": shard.hex64(digests[rank]),
                      "equal": fd == (digests[rank] & 0xFFFFFFFFFFFFFFFF)}
        entries = [shard.ShardEntry(r, *shard.shard_range(B * world, world, r), shard.hex64(d),
                                    shard.shard_file(args.out_dir, r)) for r, d in enumerate(digests)]
        if rank == 0:
            shard.write_manifest(os.path.join(args.out_dir, "trace.manifest.json"), model.name, B * world, entries)

    # ---- PCIe ceiling of this rank, measured in this run: one 1 GiB copy, and the same bytes
    # as two concurrent copies on two streams (do two SDMA engines beat one?)
    d2h_peak = d2h_probe(device)
    d2h_peak2 = d2h_probe(device, streams=2)
    if stop("d2h"):
        return 0
    trace_bytes = caps[0].layout.total
    d2h_achieved = trace_bytes / (elapsed_max / args.steps) / 1e9 if not args.no_trace else 0.0

    # ---- parity: the trace image vs the CPU oracle, record for record.  Every rank checks
    # ceil(B / N) samples spread over its shard (B samples in all, as many as at N = 1), with its
    # share of the host cores; then rank 0 alone times the CPU baseline on its NUMA node's
    # cores (capped by the cgroup quota) while the other ranks wait at a host-side barrier,
    # and checks each sample that traces as well.
    parity = Parity(read_trace(caps[0].bytes()).records) if not args.no_trace else None
    cpu = None
    quota = cpu_quota()
    host_group = dist.new_group(backend="gloo") if pg else None
    if parity is not None:
        from oracle import graph_ref
        # (at N = 1 the CPU baseline's samples are the parity set; --skip-cpu keeps two)
        n_spread = -(-B // world) if world > 1 else (2 if args.skip_cpu else 0)
        if n_spread:
            mine = os.sched_getaffinity(0)
            share = len(mine) if quota is None else max(1, min(len(mine), int(quota / world)))
            one = model_fn(batch=1)
            for i in spread_samples(count, n_spread):
                rec = graph_ref.calibrate(one.mod, one.params, {"data": x[i:i + 1]}, backend="c", threads=share)
                parity.check(i, offset + i, rec)
                del rec
        if pg:
            dist.barrier(group=host_group)
        if rank == 0 and not args.skip_cpu:
            cpus = home_cpus if world == 1 else os.sched_getaffinity(0)
            os.sched_setaffinity(0, cpus)
            threads = len(cpus) if quota is None else max(1, min(len(cpus), int(quota)))
            _log(f"cpu baseline (oracle port, {threads} threads) + parity ...")
            cpu = cpu_baseline(model_fn, offset, count, args.cpu_budget_s, threads, parity)
            cpu["n_gpus_running"] = world
        if pg:
            dist.barrier(group=host_group)
    per_step = {"min": round(min(step_gbps), 2), "max": round(max(step_gbps), 2),
                "mean": round(sum(step_gbps) / len(step_gbps), 2)} if step_gbps else None
    rank_info = {"rank": rank, "host": host_id(), "pci": placement["pci"], "numa_node": placement["numa_node"],
                 "cpus": placement["cpus"], "image_pages_per_node": image_pages,
                 "d2h": {"achieved_GBps": round(trace_bytes / (elapsed / args.steps) / 1e9, 2),
                         "measured_peak_GBps": round(d2h_peak, 2),
                         "measured_peak_2streams_GBps": round(d2h_peak2, 2),
                         "frac": round(trace_bytes / (elapsed / args.steps) / 1e9 / d2h_peak, 4),
                         "per_step_GBps": per_step},
                 "parity": parity.summary() if parity is not None else None,
                 "file_sink": file_check}
    if file_check is not None:
        # disk-write probe on the same filesystem, same writer (tk_write_file: O_DIRECT, 256 MiB
        # pieces, 2 threads), no GPU work beside it: the sink's ceiling on this box
        probe_path = path + ".probe"
        for _ in range(2):
            tp = time.perf_counter()
            caps[0].write(probe_path)
            probe_s.append(time.perf_counter() - tp)
        os.remove(probe_path)
        achieved = trace_bytes / (elapsed / args.steps) / 1e9
        probe = trace_bytes / min(probe_s) / 1e9
        file_check.update(achieved_GBps=round(achieved, 2), probe_GBps=round(probe, 2), frac=round(achieved / probe, 4),
                          probe_runs_GBps=[round(trace_bytes / t / 1e9, 2) for t in probe_s],
                          note="trace image bytes per traced step (written while the next step runs) vs the same "
                               "image written alone by the same writer, best of 2 probes before the timed region "
                               "and 2 after")
    if pg:
        ranks = [None] * world
        dist.all_gather_object(ranks, rank_info)
    else:
        ranks = [rank_info]

    rc = 0
    if rank == 0:
        traces = B * world * args.steps
        value = traces / elapsed_max
        macs_per_sample = zoo.macs_per_sample(model_fn(batch=1))
        par = None
        if parity is not None:
            ps = [r["parity"] for r in ranks]
            par = {"samples": sum(p["samples"] for p in ps), "records": sum(p["records"] for p in ps),
                   "mismatches": sum(p["mismatches"] for p in ps),
                   "first_mismatch": next((p["first_mismatch"] for p in ps if p["first_mismatch"]), None),
                   "oracle": "oracle/graph_ref.py C backend (reference int16 conv / int64 requantize semantics)"}
            rc = 1 if par["mismatches"] else 0
        if any(r.get("file_sink") and not r["file_sink"]["equal"] for r in ranks):
            _log("FILE SINK FAILURE: a written trace file's digest differs from its device digest")
            rc = 1
        line = {
            "metric": metric_for(args.model),
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
            "data": f"synthetic (seeded int8 inputs, random-init int8 weights of the "
                    f"{WORKLOADS.get(args.model, ('', args.model))[1]} topology)",
            "config": {"workload": f"{args.model} int8 224x224, {B} samples per GPU "
                                   f"({WORKLOADS.get(args.model, ('custom',))[0]}), "
                                   f"full per-op trace to pinned host memory",
                       "model": args.model, "global_batch": B * world, "samples_per_gpu": B, "seq_len": None,
                       "parallelism": f"batch-shard x{world}", "sink": args.sink,
                       "dist_backend": args.dist_backend if pg else None},
            "roofline": {"bound": "hbm", "achieved": round(achieved_bw / 1e9, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved_bw / 1e9 / HBM_PEAK_GBPS, 4),
                         "traffic": None if pmc is None else int(pmc["per_launch"]),
                         "traffic_unit": "HBM bytes per block-kernel launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                                         "per step / launches per step)",
                         "traffic_source": None if pmc is None else pmc["source"],
                         "traffic_library_match": None if pmc is None else pmc["library_match"],
                         "traffic_kernel_match": None if pmc is None else pmc["kernel_match"],
                         "traffic_bytes_per_step": None if pmc is None else int(pmc["per_step"]),
                         "launches_per_step": None if pmc is None else pmc["launches"],
                         "algorithmic_bytes_per_node": int(blk_bytes / max(n_launch, 1)),
                         "kernel": "fused conv/dense layer blocks, the find step's pick per node: conv_img_kernel "
                                   "(whole-image tiles on 28x28/14x14/7x7 planes, 3x3 split-K as a partial and an "
                                   "epilogue pass), gemm_i8_kernel<*,*,block> (im2col tiles), conv_pf_kernel "
                                   "(persistent im2col), dw_tile_kernel (depthwise 3x3 tiles on v_dot4_i32_i8, MobileNetV2), "
                                   "dense_tile_kernel (classifier); v_mfma_i32_32x32x32_i8",
                         "nodes_per_step": n_launch, "kernel_ms_per_step": round(blk_ms, 3),
                         "algorithmic_bytes_per_step": int(blk_bytes),
                         "mfma_tops": round(achieved_ops / 1e12, 1),
                         "mfma_frac": round(achieved_ops / INT8_MFMA_PEAK_OPS, 4),
                         # counted (rocprofv3, the same PMC summary as `traffic`): matrix-core busy
                         # cycles per step (SQ_VALU_MFMA_BUSY_CYCLES, summed over the 1024 SIMDs; 32 per
                         # v_mfma_i32_32x32x32_i8) over the SIMD-cycles of this run's event-timed block
                         # kernels at the 2.4 GHz peak clock; mfma_busy_gui divides by the counters' own
                         # GRBM_GUI_ACTIVE instead (rocprofiler-sdk's MfmaUtil; it also counts each
                         # dispatch's setup, so it reads lower)
                         "mfma_busy": None if pmc is None or not pmc.get("mfma") or blk_ms <= 0 else
                         round(pmc["mfma"]["SQ_VALU_MFMA_BUSY_CYCLES"] / (MFMA_SIMDS * PEAK_CLOCK_HZ * blk_ms * 1e-3), 4),
                         "mfma_busy_gui": None if pmc is None or not pmc.get("mfma") else pmc["mfma"]["mfma_busy"],
                         "mfma_counters": None if pmc is None else pmc.get("mfma"),
                         "d2h": {"achieved_GBps": round(d2h_achieved, 2), "measured_peak_GBps": round(d2h_peak, 2),
                                 "frac": round(d2h_achieved / d2h_peak, 4) if d2h_peak else None,
                                 "measured_peak_2streams_GBps": round(d2h_peak2, 2),
                                 "per_step_GBps": per_step,
                                 "note": "trace image bytes per step / max-over-ranks step time vs a 1 GiB pinned "
                                         "D2H copy measured on rank 0 in this run; per_step_GBps: record bytes per "
                                         "step over the capture stream's span (HIP events around each step's copies "
                                         "on that stream, which in the packed graph mode also waits for the first "
                                         "chunk's kernels)"}},
            "cpu_baseline": cpu,
            "parity": par,
            "file_sink": None if args.sink != "file" else
            {k: ranks[0]["file_sink"].get(k) for k in ("achieved_GBps", "probe_GBps", "frac", "equal", "overlap",
                                                      "overlap_pick_ms_per_step", "filesystem", "writer")},
            "ranks": ranks,
            "extra": {
                "compute_only_ms_per_step": round(compute_ms, 3),
                "compute_only_traces_per_s": round(B * world / (compute_ms * 1e-3), 1),
                "compute_step_device_ms": round(total_ms, 3),
                "block_segments": len(blk_segs),
                "run_mode": "hip graph per step (tk_module_run_graph)" if m.module.use_graph else
                            "host-issued kernels and copies (tk_module_run)",
                "run_mode_pick": mode_pick,
                "graph_copies": ("packed image, %d host-issued chunk copies" % args.trace_chunks
                                 if args.graph_copies == 0 else f"tk_module_set_graph_copies({args.graph_copies})")
                if m.module.use_graph else None,
                "kernels": tune_info,
                "find_step": {"tuned_nodes": len(tuning),
                              "image_tile_nodes": sum(1 for t in tuning if t["algo"] >= 16),
                              "im2col_nodes": sum(1 for t in tuning if t["algo"] == 1),
                              "persistent_nodes": sum(1 for t in tuning if t["algo"] in (3, 4)),
                              "best_us_sum": round(sum(t["us"] for t in tuning), 1)},
                "trace_bytes_per_step": trace_bytes,
                "trace_GBps_per_gpu": round(trace_bytes / (elapsed_max / args.steps) / 1e9, 2),
                "macs_per_sample": macs_per_sample,
                "ops_per_sample": 2 * macs_per_sample,
                # per-op records/s = op-traces/s x records per sample (graph inputs and
                # every op output)
                "records_per_sample": len(m.plan.records),
                "op_records_per_s": round(value * len(m.plan.records), 1),
                "record_digests": [shard.hex64(d) for d in digests],
                "collectives": {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                                "device": str(coll_dev),
                                "ran": ["barrier", "all_reduce(max elapsed)", "all_gather(record digest)",
                                        "all_gather_object(rank info)", "broadcast(status)"]} if pg else None,
                "library": _lib.build_info(),
                "host_cpus": {"affinity": len(home_cpus), "cgroup_quota": quota, "os_cpu_count": os.cpu_count()},
            },
        }
        print(json.dumps(line), flush=True)
        if rc:
            _log(f"PARITY FAILURE: {par['mismatches']} mismatching records, first {par['first_mismatch']}")
    if pg:
        flag = torch.tensor([rc], dtype=torch.int32, device=coll_dev)
        dist.broadcast(flag, 0)
        rc = int(flag.item())
        dist.destroy_process_group()
    teardown()
    return rc


if __name__ == "__main__":
    sys.exit(main())

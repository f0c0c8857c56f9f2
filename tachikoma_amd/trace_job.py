"""Resumable trace generation over a dataset larger than one batch (SURVEY.md §5,
"checkpoint / resume": the reference has no trace resume; samples are independent,
python/tvm/mrt/trace.py:65-117, so a shard is resumable per batch index).

A rank's shard of the global sample range (``shard.shard_range``) is cut into chunks of
``chunk`` samples; chunk c is traced as one batch and written to its own trace file
``<stem>.rank<r>.chunk<c>.tkt`` whose header carries the chunk's ``sample_offset``.  A
chunk counts as done only once its file is complete on disk: the file is written under a
``.partial`` name, fsync'd and renamed, and then one JSON line
``{"chunk", "sample_offset", "n_samples", "file", "bytes", "digest"}`` is appended (and
fsync'd) to the rank's journal ``<stem>.rank<r>.journal``.  A restarted job replays the
journal, keeps the chunks whose entry matches the plan and whose file still has the
recorded size (and, with ``verify``, the recorded record digest), and traces the rest.  A
crash at any point therefore loses at most the chunks in flight.

On the device the chunk files are produced by :class:`GraphModuleTracer`: two pinned trace
images alternate, so chunk c's file is written by a host thread while chunk c+1 runs and
its records are copied D2H (the bench's file sink, overlapped with the next batch).

CLI (one process per GPU, torch.distributed.run environment; rank 0 writes the manifest)::

    python -m tachikoma_amd.trace_job --model resnet50 --samples 4096 --chunk 64 --out-dir DIR
"""
from __future__ import annotations

import argparse
import concurrent.futures
import json
import os
import sys
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

from . import shard
from . import trace_format as tf

JOURNAL_FORMAT = "tachikoma-trace-journal"


@dataclass(frozen=True)
class Chunk:
    index: int
    sample_offset: int
    n_samples: int
    file: str


def chunk_file(out_dir: str, rank: int, index: int, stem: str = "trace") -> str:
    return os.path.join(out_dir, f"{stem}.rank{rank}.chunk{index}.tkt")


def journal_file(out_dir: str, rank: int, stem: str = "trace") -> str:
    return os.path.join(out_dir, f"{stem}.rank{rank}.journal")


def plan_chunks(global_samples: int, world: int, rank: int, chunk: int, out_dir: str,
                stem: str = "trace") -> List[Chunk]:
    """This rank's contiguous shard cut into chunks of ``chunk`` samples (the last one may be
    shorter); chunk indices are per rank."""
    if chunk <= 0:
        raise ValueError("chunk must be positive")
    off, n = shard.shard_range(global_samples, world, rank)
    out = []
    for i, s in enumerate(range(0, n, chunk)):
        out.append(Chunk(i, off + s, min(chunk, n - s), chunk_file(out_dir, rank, i, stem)))
    return out


def _fsync_dir(path: str) -> None:
    try:
        fd = os.open(os.path.dirname(os.path.abspath(path)) or ".", os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


class Journal:
    """Append-only JSON-lines record of the chunks whose files are complete."""

    def __init__(self, path: str):
        self.path = path

    def entries(self) -> Dict[int, dict]:
        """chunk index → last entry; a torn last line (crash during append) is ignored."""
        out: Dict[int, dict] = {}
        try:
            with open(self.path) as f:
                lines = f.read().split("\n")
        except FileNotFoundError:
            return out
        for ln in lines:
            if not ln.strip():
                continue
            try:
                e = json.loads(ln)
            except json.JSONDecodeError:
                continue
            if e.get("format") == JOURNAL_FORMAT and isinstance(e.get("chunk"), int):
                out[e["chunk"]] = e
        return out

    def append(self, entry: dict) -> None:
        line = json.dumps(dict(entry, format=JOURNAL_FORMAT), separators=(",", ":")) + "\n"
        with open(self.path, "a") as f:
            f.write(line)
            f.flush()
            os.fsync(f.fileno())

    def reset(self) -> None:
        if os.path.exists(self.path):
            os.remove(self.path)


def _valid(entry: dict, c: Chunk, verify: bool) -> bool:
    if (entry.get("sample_offset"), entry.get("n_samples"), entry.get("file")) != (c.sample_offset, c.n_samples,
                                                                                     os.path.basename(c.file)):
        return False
    try:
        if os.path.getsize(c.file) != entry.get("bytes"):
            return False
    except OSError:
        return False
    if verify:
        try:
            return shard.hex64(tf.trace_file_digest(c.file)) == entry.get("digest")
        except (OSError, ValueError):
            return False
    return True


# A tracer takes (sample_offset, n_samples, path) and returns a Future that resolves to the
# u64 record digest once ``path`` holds the complete trace file of those samples.
Tracer = Callable[[int, int, str], "concurrent.futures.Future[int]"]


def run(tracer: Tracer, global_samples: int, chunk: int, out_dir: str, rank: int = 0, world: int = 1,
        resume: bool = True, verify: bool = False, stem: str = "trace",
        log: Optional[Callable[[str], None]] = None) -> List[shard.ShardEntry]:
    """Trace this rank's chunks that are not done yet; returns the entries of ALL its chunks
    (resumed and new) in sample order."""
    os.makedirs(out_dir, exist_ok=True)
    chunks = plan_chunks(global_samples, world, rank, chunk, out_dir, stem)
    journal = Journal(journal_file(out_dir, rank, stem))
    if not resume:
        journal.reset()
    done = journal.entries() if resume else {}
    kept = {c.index: done[c.index] for c in chunks if c.index in done and _valid(done[c.index], c, verify)}
    todo = [c for c in chunks if c.index not in kept]
    if log:
        log(f"rank {rank}: {len(chunks)} chunks, {len(kept)} done, {len(todo)} to trace")
    pending: List = []

    def finish(c: Chunk, fut) -> None:
        digest = int(fut.result()) & 0xFFFFFFFFFFFFFFFF
        tmp = c.file + ".partial"
        with open(tmp, "rb+") as f:
            os.fsync(f.fileno())
        os.replace(tmp, c.file)
        _fsync_dir(c.file)
        e = {"chunk": c.index, "sample_offset": c.sample_offset, "n_samples": c.n_samples,
             "file": os.path.basename(c.file), "bytes": os.path.getsize(c.file), "digest": shard.hex64(digest)}
        journal.append(e)
        kept[c.index] = e

    for c in todo:
        try:
            fut = tracer(c.sample_offset, c.n_samples, c.file + ".partial")
        except BaseException:
            # chunks already handed to the tracer still complete: journal those whose files do
            # before the failure propagates (a resume then re-traces only what was lost)
            for pc, pf in pending:
                try:
                    finish(pc, pf)
                except Exception:  # noqa: BLE001 - the original failure is the one to report
                    break
            raise
        pending.append((c, fut))
        # journal entries are appended in chunk order, as soon as each file is complete
        while pending and (len(pending) > 1 or pending[0][1].done()):
            finish(*pending.pop(0))
    while pending:
        finish(*pending.pop(0))
    return [shard.ShardEntry(rank, c.sample_offset, c.n_samples, kept[c.index]["digest"], kept[c.index]["file"])
            for c in chunks]


class GraphModuleTracer:
    """Device tracer over built GraphModules (one per distinct chunk size): chunk c's pinned
    image is written to its file by a writer thread while chunk c+1 runs on the GPU."""

    def __init__(self, build_module: Callable[[int], "object"], inputs: Callable[[int, int], "object"],
                 model: str = "graph", input_name: str = "data", rank: int = 0, world: int = 1):
        self.build_module = build_module
        self.inputs = inputs
        self.model, self.input_name, self.rank, self.world = model, input_name, rank, world
        self.modules: Dict[int, list] = {}  # n_samples -> [GraphModule, [TraceCapture x2], next slot]
        self.writer = concurrent.futures.ThreadPoolExecutor(max_workers=1)
        self.busy: Dict[int, "concurrent.futures.Future"] = {}
        self.digest_slots: Dict[int, "object"] = {}  # per trace image: pinned host copy of its digest

    def _module(self, n: int):
        if n not in self.modules:
            from .contrib.graph_executor import TraceCapture
            m = self.build_module(n)
            # traced runs as one replayed HIP graph: one host call per chunk, so a host that issues
            # calls late cannot starve the copies (profiles/r03r_run_modes_slow_host.txt)
            m.module.use_graph = True
            caps = [m.trace_capture(), TraceCapture(m.module, m._meta)]
            self.modules[n] = [m, caps, 0]
        return self.modules[n]

    def __call__(self, sample_offset: int, n_samples: int, path: str):
        import torch
        entry = self._module(n_samples)
        m, caps, slot = entry
        cap = caps[slot]
        entry[2] = 1 - slot
        prev = self.busy.get(id(cap))
        if prev is not None:
            prev.result()  # the writer is done with this image
        meta = dict(model=self.model, sample_offset=sample_offset, n_samples=n_samples, rank=self.rank,
                    world=self.world)
        m._meta.update(meta)
        cap.update_meta(**meta)
        m.set_input(self.input_name, self.inputs(sample_offset, n_samples))
        stream = torch.cuda.current_stream(m.module.device)
        cap.capture_inputs(stream)
        m.module.run(stream, cap.capture_stream, cap.host_dst)
        # device digest of exactly these records, copied on the stream into this image's own
        # pinned slot: the module's digest tensor is reused by the next chunk's run, which the
        # stream may reach before the writer thread reads the value
        digest = m.module.records_digest(stream)
        slot_t = self.digest_slots.get(id(cap))
        if slot_t is None:
            slot_t = self.digest_slots[id(cap)] = torch.empty(digest.shape, dtype=digest.dtype, pin_memory=True)
        slot_t.copy_(digest, non_blocking=True)
        done = torch.cuda.Event()
        done.record(stream)

        def write() -> int:
            done.synchronize()
            cap.synchronize()
            cap.write(path)
            return int(slot_t.reshape(-1)[0].item()) & 0xFFFFFFFFFFFFFFFF

        fut = self.writer.submit(write)
        self.busy[id(cap)] = fut
        return fut

    def close(self) -> None:
        """Wait for the writer, then release every module (device first, then the native module:
        GraphModule.close) while the HIP runtime is alive."""
        self.writer.shutdown(wait=True)
        for m, caps, _ in self.modules.values():
            m.close()
            caps.clear()
        self.modules.clear()
        self.digest_slots.clear()


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--model", default="resnet50")
    p.add_argument("--samples", type=int, required=True, help="global number of samples")
    p.add_argument("--chunk", type=int, default=64, help="samples per chunk (one traced batch)")
    p.add_argument("--out-dir", required=True)
    p.add_argument("--no-resume", action="store_true", help="start over (drop the journal)")
    p.add_argument("--verify", action="store_true", help="re-digest resumed chunk files")
    args = p.parse_args(argv)
    import torch
    from . import relay, zoo
    from .contrib import graph_executor
    rank, world, local = shard.dist_env()
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # manifest exchange only; no data-path collective
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    model_fn = zoo.MODELS[args.model]
    proto = model_fn(batch=1)

    def build_module(n: int):
        mdl = model_fn(batch=n)
        lib = relay.build(mdl.mod, target="mi355x", params=mdl.params)
        return graph_executor.GraphModule(lib["default"](device.index))

    tracer = GraphModuleTracer(build_module, proto.sample_inputs, model=proto.name, input_name=proto.input_name,
                               rank=rank, world=world)
    log = lambda s: print(f"[trace_job] {s}", file=sys.stderr, flush=True)  # noqa: E731
    try:
        entries = run(tracer, args.samples, args.chunk, args.out_dir, rank, world, resume=not args.no_resume,
                      verify=args.verify, log=log)
    finally:
        tracer.close()
    if world > 1:
        import torch.distributed as dist
        allents: List = [None] * world
        dist.all_gather_object(allents, entries)
        entries = [e for es in allents for e in es]
        dist.destroy_process_group()
    if rank == 0:
        path = os.path.join(args.out_dir, "trace.manifest.json")
        shard.write_manifest(path, proto.name, args.samples, entries, world=world)
        log(f"manifest {path}: {len(entries)} chunks")
    return 0


if __name__ == "__main__":
    sys.exit(main())

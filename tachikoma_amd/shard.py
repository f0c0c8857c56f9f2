"""Batch sharding of trace generation across the GPUs of one node.

Every sample's trace is independent (the reference walks one sample at a time with
no cross-sample state, python/tvm/mrt/trace.py:65-117), so the global batch is cut
into contiguous shards, one per rank (one process per GPU), with no collective on
the data path.  Each rank writes its own trace file whose header carries
``sample_offset``; the only collective is an optional all-gather of one u64 record
digest per rank (RCCL over xGMI when the tensors live on the GPU, gloo on CPU) so
rank 0 can write a run manifest that pins every shard.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass
from typing import List, Optional, Tuple

MANIFEST_FORMAT = "tachikoma-trace-manifest"


def shard_range(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """(sample_offset, n_samples) of ``rank``: contiguous, remainder to the first ranks."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    if global_batch < 0:
        raise ValueError("negative batch")
    base, rem = divmod(global_batch, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def dist_env() -> Tuple[int, int, int]:
    """(rank, world, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _to_i64(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= 1 << 63 else v


def gather_digests(digest, device=None) -> List[int]:
    """All-gather one u64 per rank over the default process group.

    ``digest`` is an int or a 1-element int64 tensor (e.g. DeviceModule.records_digest,
    already on the GPU so RCCL moves it over xGMI without a host round trip)."""
    import torch
    import torch.distributed as dist
    if isinstance(digest, torch.Tensor):
        t = digest.reshape(1).to(torch.int64)
    else:
        t = torch.tensor([_to_i64(int(digest))], dtype=torch.int64, device=device)
    if not (dist.is_available() and dist.is_initialized()):
        return [int(t.item()) & 0xFFFFFFFFFFFFFFFF]
    # (at world size 1 the all-gather still runs: bench.py --force-pg exercises the RCCL path)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [int(v.item()) & 0xFFFFFFFFFFFFFFFF for v in out]


def shard_file(out_dir: str, rank: int, stem: str = "trace") -> str:
    return os.path.join(out_dir, f"{stem}.rank{rank}.tkt")


@dataclass
class ShardEntry:
    rank: int
    sample_offset: int
    n_samples: int
    digest: str  # u64 as 16 hex digits
    file: Optional[str] = None


def write_manifest(path: str, model: str, global_batch: int, shards: List[ShardEntry],
                   world: Optional[int] = None) -> None:
    """Run manifest: every shard (or chunk of a shard, see trace_job) with its sample range,
    u64 record digest and file; the entries must tile [0, global_batch) exactly."""
    covered = sorted((s.sample_offset, s.n_samples) for s in shards)
    pos = 0
    for off, n in covered:
        if off != pos:
            raise ValueError(f"shards do not tile the batch: gap/overlap at sample {pos}")
        pos += n
    if pos != global_batch:
        raise ValueError(f"shards cover {pos} of {global_batch} samples")
    doc = {"format": MANIFEST_FORMAT, "version": 1, "model": model, "global_batch": global_batch,
           "world": len(shards) if world is None else int(world),
           "shards": [asdict(s) for s in sorted(shards, key=lambda s: (s.rank, s.sample_offset))]}
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(doc, f, indent=1)
    os.replace(tmp, path)


def read_manifest(path: str) -> dict:
    with open(path) as f:
        doc = json.load(f)
    if doc.get("format") != MANIFEST_FORMAT:
        raise ValueError("not a tachikoma trace manifest")
    return doc


def hex64(v: int) -> str:
    return f"{v & 0xFFFFFFFFFFFFFFFF:016x}"


# ---------------------------------------------------------------- host placement
# Each rank pins a whole shard image (7.45 GB for ResNet-50 at 64 samples) that its GPU
# writes at PCIe rate; at 8 GPUs that is ~450 GB/s of host writes, so every image must sit
# in the DRAM of its GPU's own socket.  The rank binds itself to the CPUs of the GPU's NUMA
# node before allocating (pinned pages are placed by the allocating thread's node under the
# default local policy) and reports where the pages landed.

def gpu_pci_address(device_index: int) -> Optional[str]:
    """PCI address (domain:bus:device.function) of a visible GPU, from the HIP runtime."""
    import torch
    p = torch.cuda.get_device_properties(device_index)
    try:
        return f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}.0"
    except AttributeError:
        return None


SYSFS = os.environ.get("TK_SYSFS_ROOT", "/sys")  # a fake tree in tests (tests/test_placement.py)


def pci_numa_node(pci: Optional[str], sysfs: Optional[str] = None) -> Optional[int]:
    if not pci:
        return None
    try:
        with open(f"{sysfs or SYSFS}/bus/pci/devices/{pci}/numa_node") as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        return None
    return node if node >= 0 else None


def _parse_cpulist(text: str) -> List[int]:
    cpus: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def node_cpus(node: int, sysfs: Optional[str] = None) -> List[int]:
    try:
        with open(f"{sysfs or SYSFS}/devices/system/node/node{node}/cpulist") as f:
            return _parse_cpulist(f.read())
    except OSError:
        return []


def placement(pci: Optional[str], affinity=None, sysfs: Optional[str] = None) -> dict:
    """Where a rank driving the GPU at ``pci`` runs: the GPU's NUMA node and that node's CPUs
    within ``affinity`` (default: this process's).  Pure: nothing is bound.  {"pci", "numa_node",
    "cpus" (sorted list), "bound"}: bound is False (cpus = affinity) when the node or its CPU list
    cannot be read or does not meet the affinity."""
    aff = sorted(os.sched_getaffinity(0) if affinity is None else affinity)
    node = pci_numa_node(pci, sysfs)
    cpus = sorted(set(node_cpus(node, sysfs)) & set(aff)) if node is not None else []
    return {"pci": pci, "numa_node": node, "cpus": cpus or aff, "bound": bool(cpus)}


def rank_plan(world: int, pcis: List[Optional[str]], affinity=None, sysfs: Optional[str] = None) -> List[dict]:
    """The N-rank launch plan of one node (bench.py --gpus N, one process per GPU): rank r drives
    GPU r (LOCAL_RANK = r), binds to its GPU's NUMA node's CPUs and first-touches its pinned trace
    image from there, so every image sits in its own socket's DRAM.  Fails when there are fewer
    GPUs than ranks (one GPU per rank)."""
    if world > len(pcis):
        raise ValueError(f"{world} ranks need {world} GPUs, {len(pcis)} visible")
    return [dict(rank=r, gpu=r, image_node=p["numa_node"], **p)
            for r, p in ((r, placement(pcis[r], affinity, sysfs)) for r in range(world))]


def bind_to_gpu_node(device_index: int, pci: Optional[str] = None, sysfs: Optional[str] = None) -> dict:
    """Restrict this process to the CPUs of the GPU's NUMA node (intersected with the current
    affinity).  Returns {"pci", "numa_node", "cpus" (count), "bound"}; nothing changes when the
    node or its CPU list cannot be read."""
    info = placement(pci if pci is not None else gpu_pci_address(device_index), sysfs=sysfs)
    if info["bound"]:
        os.sched_setaffinity(0, info["cpus"])
    return dict(info, cpus=len(info["cpus"]))


def numa_pages(ptr: int, nbytes: int) -> Optional[dict]:
    """{node: pages} of the mappings overlapping [ptr, ptr + nbytes) from /proc/self/numa_maps
    (None where the kernel does not expose it)."""
    try:
        with open("/proc/self/maps") as f:
            ranges = {}
            for line in f:
                lo, hi = (int(x, 16) for x in line.split()[0].split("-"))
                if lo < ptr + nbytes and hi > ptr:
                    ranges[lo] = hi
        out: dict = {}
        with open("/proc/self/numa_maps") as f:
            for line in f:
                fields = line.split()
                if int(fields[0], 16) not in ranges:
                    continue
                for fld in fields[1:]:
                    if fld.startswith("N") and "=" in fld:
                        k, v = fld[1:].split("=")
                        out[int(k)] = out.get(int(k), 0) + int(v)
        return out or None
    except (OSError, ValueError):
        return None

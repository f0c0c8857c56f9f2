"""The 8-rank launch / placement plan on a faked two-socket topology (CPU only):
rank -> GPU -> NUMA node -> CPUs, and the pinned trace image first-touched from the rank's node.
The topology is a fake sysfs tree (TK_SYSFS_ROOT): 8 GPUs, 4 per node, node 0 owning CPUs 0-3
and node 1 CPUs 4-7 of this container, so real processes can bind to them."""
import json
import os
import subprocess
import sys

import pytest

from tachikoma_amd import shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PCIS = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xe5, 0xf5)]


@pytest.fixture
def fake_sysfs(tmp_path):
    aff = sorted(os.sched_getaffinity(0))
    if len(aff) < 2:
        pytest.skip("needs two CPUs to fake two nodes")
    half = len(aff) // 2
    nodes = {0: aff[:half], 1: aff[half:]}
    for i, pci in enumerate(PCIS):
        d = tmp_path / "bus" / "pci" / "devices" / pci
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{i // 4}\n")
    for n, cpus in nodes.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(",".join(str(c) for c in cpus) + "\n")
    return str(tmp_path), nodes


def test_rank_plan_two_sockets(fake_sysfs):
    root, nodes = fake_sysfs
    plan = shard.rank_plan(8, PCIS, sysfs=root)
    assert [p["gpu"] for p in plan] == list(range(8))  # one GPU per rank
    assert [p["numa_node"] for p in plan] == [0] * 4 + [1] * 4
    for p in plan:
        assert p["bound"] and p["cpus"] == nodes[p["numa_node"]]
        assert p["image_node"] == p["numa_node"]  # first touch from the GPU's own socket
    # 4 ranks share each socket's CPUs (and its DRAM write bandwidth)
    assert sum(p["numa_node"] == 0 for p in plan) == 4


def test_rank_plan_edge_cases(fake_sysfs, tmp_path):
    root, nodes = fake_sysfs
    with pytest.raises(ValueError):
        shard.rank_plan(9, PCIS, sysfs=root)
    # unknown GPU / missing node / affinity outside the node: unbound, keeps the affinity
    p = shard.placement("ffff:ff:1f.7", affinity=[0, 1], sysfs=root)
    assert not p["bound"] and p["numa_node"] is None and p["cpus"] == [0, 1]
    p = shard.placement(PCIS[7], affinity=nodes[0], sysfs=root)
    assert p["numa_node"] == 1 and not p["bound"] and p["cpus"] == nodes[0]


_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["TK_ROOT"])
import numpy as np
from tachikoma_amd import shard
rank = int(os.environ["RANK"])
pcis = os.environ["TK_PCIS"].split(",")
info = shard.bind_to_gpu_node(int(os.environ["LOCAL_RANK"]), pci=pcis[int(os.environ["LOCAL_RANK"])])
img = np.zeros(8 << 20, np.uint8)
img[::4096] = 1  # first touch from the bound CPUs
out = dict(info, rank=rank, world=int(os.environ["WORLD_SIZE"]), affinity=sorted(os.sched_getaffinity(0)),
           pages=shard.numa_pages(img.ctypes.data, img.nbytes))
with open(os.path.join(os.environ["TK_OUT"], f"rank{rank}.json"), "w") as f:
    json.dump(out, f)
"""


def test_launch_eight_ranks_binds_each_to_its_node(fake_sysfs, tmp_path):
    """bench.launch_ranks starts 8 real processes (RANK = LOCAL_RANK = r, WORLD_SIZE 8); each binds
    itself through shard.bind_to_gpu_node to its GPU's node and first-touches an image there."""
    root, nodes = fake_sysfs
    import bench
    out = tmp_path / "out"
    out.mkdir()
    script = tmp_path / "child.py"
    script.write_text(_CHILD)
    env = dict(os.environ, TK_SYSFS_ROOT=root, TK_PCIS=",".join(PCIS), TK_OUT=str(out), TK_ROOT=ROOT)
    old = dict(os.environ)
    os.environ.update(env)
    try:
        rc = bench.launch_ranks(8, [sys.executable, str(script)])
    finally:
        os.environ.clear()
        os.environ.update(old)
    assert rc == 0
    got = [json.loads((out / f"rank{r}.json").read_text()) for r in range(8)]
    for r, g in enumerate(got):
        node = r // 4
        assert g["rank"] == r and g["world"] == 8 and g["numa_node"] == node and g["bound"]
        assert g["affinity"] == nodes[node] and g["cpus"] == len(nodes[node])
        assert g["pages"] is None or sum(g["pages"].values()) > 0

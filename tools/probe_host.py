"""Host facts of a GPU box: CPUs visible vs granted, NUMA nodes, GPU PCI address / node."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tachikoma_amd import shard  # noqa: E402

info = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_quota": bench.cpu_quota(),
        "env": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "MAX_JOBS", "HIP_VISIBLE_DEVICES")}}
nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit())
info["numa_nodes"] = {n: len(shard.node_cpus(n)) for n in nodes}
import torch  # noqa: E402
info["gpus"] = []
for i in range(torch.cuda.device_count()):
    pci = shard.gpu_pci_address(i)
    info["gpus"].append({"index": i, "pci": pci, "numa_node": shard.pci_numa_node(pci)})
try:
    with open("/proc/meminfo") as f:
        info["mem_total_kb"] = int(f.readline().split()[1])
except OSError:
    pass
print(json.dumps(info))

"""The RCCL branch of bench.py on the one GPU a box has: a child process starts a
world-size-1 ``nccl`` process group before any GPU call (bench.py --force-pg), runs every
collective the N>1 path uses -- barrier, the elapsed-time all_reduce(MAX), the device record-digest
all_gather over RCCL, all_gather_object of the rank info, the status broadcast -- and writes its
shard file and manifest; the manifest's digest must equal both the digest of the written file and
the digest the all_gather returned."""
import json
import os
import subprocess
import sys

import pytest

from tachikoma_amd import shard
from tachikoma_amd.trace_format import trace_file_digest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_world1_nccl_collectives(tmp_path):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-pg", "--dist-backend", "nccl",
           "--model", "lenet5", "--batch", "8", "--steps", "2", "--warmup", "1", "--skip-cpu", "--tune-table", "none",
           "--sink", "file", "--file-overlap", "off", "--out-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    coll = line["extra"]["collectives"]
    assert coll["backend"] == "nccl" and coll["world_size"] == 1 and coll["device"].startswith("cuda")
    assert line["config"]["dist_backend"] == "nccl" and line["n_gpus"] == 1
    assert line["parity"]["mismatches"] == 0 and line["parity"]["records"] > 0
    assert line["file_sink"]["equal"] is True
    man = shard.read_manifest(str(tmp_path / "trace.manifest.json"))
    (entry,) = man["shards"]
    assert entry["rank"] == 0 and entry["sample_offset"] == 0 and entry["n_samples"] == 8
    assert entry["digest"] == line["extra"]["record_digests"][0]
    assert entry["digest"] == shard.hex64(trace_file_digest(entry["file"]))

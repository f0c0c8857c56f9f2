"""Host logic of bench.py that needs no GPU: the N-rank self-launcher (`python bench.py --gpus
N` must start N ranks, not one), the record-by-record parity checker, host placement helpers,
and a 2-rank gloo rendezvous through the launcher's environment."""
import json
import os
import sys

import numpy as np
import pytest

import bench
from tachikoma_amd import shard


def test_launcher_starts_n_ranks(tmp_path):
    out = tmp_path / "ranks"
    out.mkdir()
    code = ("import json, os, sys; d = {k: os.environ[k] for k in "
            "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}; "
            f"open(os.path.join({str(out)!r}, 'r' + d['RANK']), 'w').write(json.dumps(d))")
    assert bench.launch_ranks(3, [sys.executable, "-c", code]) == 0
    docs = [json.loads((out / f"r{r}").read_text()) for r in range(3)]
    assert [d["RANK"] for d in docs] == ["0", "1", "2"]
    assert all(d["WORLD_SIZE"] == "3" and d["MASTER_ADDR"] == "127.0.0.1" for d in docs)
    assert len({d["MASTER_PORT"] for d in docs}) == 1


def test_launcher_propagates_failure():
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(7) if r == 1 else time.sleep(60)"
    assert bench.launch_ranks(2, [sys.executable, "-c", code]) == 7  # rank 0 is terminated, not waited for


def test_launcher_gloo_rendezvous(tmp_path):
    """The launched ranks form a torch.distributed group (gloo on CPU, world 2)."""
    out = tmp_path / "sum"
    code = ("import os, torch, torch.distributed as dist; dist.init_process_group('gloo'); "
            "t = torch.tensor([dist.get_rank() + 1]); dist.all_reduce(t); "
            f"open({str(out)!r} + os.environ['RANK'], 'w').write(str(int(t)))")
    assert bench.launch_ranks(2, [sys.executable, "-c", code]) == 0
    assert [open(f"{out}{r}").read() for r in range(2)] == ["3", "3"]


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 4"):
        bench.main(["--gpus", "4", "--dist-backend", "gloo"])


def test_more_gpus_than_visible_fails_before_any_rank(monkeypatch):
    """--gpus N over RCCL with fewer visible GPUs stops at once with a clear message, before the
    launcher starts ranks or init_process_group("nccl") could wait for a missing one."""
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    started = []
    monkeypatch.setattr(bench, "launch_ranks", lambda n, cmd: started.append(n) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit, match="--gpus 8 needs 8 visible GPUs.*shows 1"):
        bench.main(["--gpus", "8"])
    monkeypatch.setenv("WORLD_SIZE", "8")
    with pytest.raises(SystemExit, match="needs 8 visible GPUs"):
        bench.main(["--gpus", "8"])
    assert started == []
    # gloo rehearses N ranks on one GPU: the launcher runs
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.main(["--gpus", "2", "--dist-backend", "gloo"]) == 0 and started == [2]


def test_parity_checker():
    rec = {"data": np.arange(12, dtype=np.int8).reshape(3, 4), "%0": np.arange(6, dtype=np.int32).reshape(3, 2)}
    p = bench.Parity(rec)
    p.check(1, 101, {"data": rec["data"][1:2].copy(), "%0": rec["%0"][1:2].copy()})
    assert p.summary() == {"samples": 1, "records": 2, "mismatches": 0, "first_mismatch": None}
    bad = rec["%0"][2:3].copy()
    bad[0, 1] += 1
    p.check(2, 102, {"%0": bad})
    s = p.summary()
    assert s["mismatches"] == 1 and s["first_mismatch"] == {"sample": 102, "record": "%0", "index": [1],
                                                            "gpu": 5, "cpu": 6}


def test_host_placement_helpers():
    assert shard._parse_cpulist("0-2,5,7-8\n") == [0, 1, 2, 5, 7, 8]
    assert shard.pci_numa_node(None) is None
    assert shard.pci_numa_node("ffff:ff:1f.7") is None
    a = np.ones(1 << 24, np.uint8)
    pages = shard.numa_pages(a.ctypes.data, a.nbytes)
    assert pages is None or sum(pages.values()) >= (1 << 24) // 4096
    q = bench.cpu_quota()
    assert q is None or q > 0


def test_parity_counts_a_rechecked_sample_once():
    rec = {"%0": np.arange(6, dtype=np.int32).reshape(3, 2)}
    p = bench.Parity(rec)
    p.check(0, 0, {"%0": rec["%0"][0:1].copy()})
    p.check(0, 0, {"%0": rec["%0"][0:1].copy()})  # the CPU baseline traces a spread sample again
    p.check(2, 2, {"%0": rec["%0"][2:3].copy()})
    assert p.summary()["samples"] == 2 and p.summary()["records"] == 2


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_parity_spread_covers_the_n1_sample_count(world):
    """ceil(64 / N) samples per rank over N shards of 64 = at least the 64 samples of N = 1,
    each rank's first and last sample included."""
    per_rank = bench.spread_samples(64, -(-64 // world))
    assert len(per_rank) * world >= 64 and per_rank[0] == 0 and per_rank[-1] == 63
    assert len(set(per_rank)) == len(per_rank)


def test_pmc_traffic_picks_library_then_stamp(tmp_path, monkeypatch):
    """bench.pmc_traffic: the summary taken with the loaded library wins; failing that the
    newest by embedded UTC stamp (not by file name); traffic per launch divides by the PMC's
    own dispatch count."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"model": "resnet50", "batch": 64, "launches_per_step": 55}

    def put(name, **kw):
        (prof / name).write_text(json.dumps(dict(base, **kw)))

    put("r09_pmc_block.json", hbm_bytes_per_step=110.0, created_utc="2026-01-01T00:00:00Z", library="old")
    put("r02z_pmc_block.json", hbm_bytes_per_step=220.0, created_utc="2026-02-01T00:00:00Z", library="older")
    put("r00_pmc_block.json", hbm_bytes_per_step=330.0)  # no stamp: never chosen
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got = bench.pmc_traffic("resnet50", 64, "current")
    assert got["source"] == os.path.join("profiles", "r02z_pmc_block.json") and not got["library_match"]
    assert got["per_launch"] == 4.0 and got["launches"] == 55
    put("r01_pmc_block.json", hbm_bytes_per_step=55.0, created_utc="2025-01-01T00:00:00Z", library="current")
    got = bench.pmc_traffic("resnet50", 64, "current")
    assert got["source"] == os.path.join("profiles", "r01_pmc_block.json") and got["library_match"]
    assert got["per_launch"] == 1.0
    assert bench.pmc_traffic("resnet18", 64, "current") is None


def test_file_sink_overlap_pick():
    """The r05r box: on / off rounds 860 / 985, 817 / 608, 555 / 606 ms per step -- a median over
    all rounds picked "off" (frac 0.77 where overlap reached 0.90); without the first round the
    later rounds decide."""
    import bench
    r05r = bench.pick_overlap({"on": [860.4, 817.3, 554.9, 550.0, 548.0], "off": [985.5, 607.9, 606.0, 605.0, 607.0]})
    assert r05r["pick"] == "on" and r05r["on"] < r05r["off"]
    r05q = bench.pick_overlap({"on": [647.1, 539.9, 546.4, 541.0, 543.0], "off": [586.8, 589.6, 589.4, 588.0, 590.0]})
    assert r05q["pick"] == "on"
    slow_disk = bench.pick_overlap({"on": [700.0, 690.0, 705.0, 698.0, 702.0], "off": [650.0, 640.0, 655.0, 645.0, 650.0]})
    assert slow_disk["pick"] == "off"
    assert bench.pick_overlap({"on": [500.0], "off": [600.0]})["pick"] == "on"

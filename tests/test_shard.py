"""Batch sharding, record digests and the run manifest.

The multi-process test runs world_size 2 over gloo on the CPU: each rank traces
its shard with the oracle (the device is not needed to check the host logic),
digests its records with the host twin of tk_digest_bytes, all-gathers the
digests through ``shard.gather_digests`` and rank 0 writes the manifest.
"""
import json
import os
import socket

import numpy as np
import pytest

from tachikoma_amd import shard, zoo
from tachikoma_amd import trace_format as tf


@pytest.mark.parametrize("batch,world", [(512, 8), (64, 1), (7, 3), (2, 4), (0, 2), (513, 8)])
def test_shard_range_tiles_batch(batch, world):
    pos = 0
    for r in range(world):
        off, n = shard.shard_range(batch, world, r)
        assert off == pos and n >= 0
        pos += n
    assert pos == batch
    counts = [shard.shard_range(batch, world, r)[1] for r in range(world)]
    assert max(counts) - min(counts) <= 1


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard.shard_range(8, 2, 2)
    with pytest.raises(ValueError):
        shard.shard_range(8, 0, 0)


def test_sample_inputs_independent_of_split():
    m = zoo.lenet5(batch=1)
    full = m.sample_inputs(0, 6)
    parts = [m.sample_inputs(*shard.shard_range(6, 4, r)) for r in range(4)]
    np.testing.assert_array_equal(np.concatenate(parts), full)
    assert full.dtype == np.int8 and full.shape == (6, 1, 28, 28)


def test_digest_known_values():
    assert tf.digest_bytes(b"") == 0
    # one word: mix64(w ^ 0) ; the same bytes at word 1 mix with φ
    a = tf.digest_bytes(np.arange(8, dtype=np.uint8).tobytes())
    b = tf.digest_bytes(np.concatenate([np.zeros(8, np.uint8), np.arange(8, dtype=np.uint8)]).tobytes())
    assert a != b
    # tail padding: a 3-byte buffer equals its zero-padded 8-byte word
    assert tf.digest_bytes(b"abc") == tf.digest_bytes(b"abc" + b"\0" * 5)
    # chunking does not change the sum
    x = np.random.default_rng(0).integers(0, 256, size=100_003, dtype=np.uint8)
    assert tf.digest_bytes(x, chunk_words=7) == tf.digest_bytes(x)


def test_digest_matches_scalar_definition():
    def mix(z):
        m = (1 << 64) - 1
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        return z ^ (z >> 31)
    data = bytes(np.random.default_rng(1).integers(0, 256, size=45, dtype=np.uint8))
    padded = data + b"\0" * (-len(data) % 8)
    want = 0
    for i in range(len(padded) // 8):
        w = int.from_bytes(padded[8 * i:8 * i + 8], "little")
        want = (want + mix(w ^ ((i * 0x9E3779B97F4A7C15) & ((1 << 64) - 1)))) & ((1 << 64) - 1)
    assert tf.digest_bytes(data) == want


def test_manifest_roundtrip_and_tiling(tmp_path):
    e = [shard.ShardEntry(0, 0, 3, "00" * 8, "a"), shard.ShardEntry(1, 3, 2, "11" * 8, "b")]
    p = str(tmp_path / "m.json")
    shard.write_manifest(p, "lenet5", 5, e)
    doc = shard.read_manifest(p)
    assert doc["world"] == 2 and doc["shards"][1]["sample_offset"] == 3
    with pytest.raises(ValueError):
        shard.write_manifest(p, "lenet5", 6, e)
    with pytest.raises(ValueError):
        shard.write_manifest(p, "lenet5", 5, [e[0], shard.ShardEntry(1, 4, 1, "0" * 16)])


def test_gather_digests_single_process():
    assert shard.gather_digests(0xFFFFFFFFFFFFFFFF) == [0xFFFFFFFFFFFFFFFF]


def _ordered_records(model, recs):
    names = [model.input_name] + [k for k in recs if k != model.input_name]
    return {k: recs[k] for k in names}


def _rank_main(rank, world, port, global_batch, out_dir):
    import torch.distributed as dist
    from oracle import graph_ref
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = zoo.lenet5(batch=1)
        off, n = shard.shard_range(global_batch, world, rank)
        x = model.sample_inputs(off, n)
        recs = _ordered_records(model, graph_ref.calibrate(model.mod, model.params, {"data": x}, threads=1))
        d = tf.records_digest(recs)
        digests = shard.gather_digests(d)
        assert digests[rank] == d
        if rank == 0:
            entries = [shard.ShardEntry(r, *shard.shard_range(global_batch, world, r), shard.hex64(v))
                       for r, v in enumerate(digests)]
            shard.write_manifest(os.path.join(out_dir, "manifest.json"), model.name, global_batch, entries)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_digest_manifest(tmp_path):
    import torch.multiprocessing as mp
    from oracle import graph_ref
    world, global_batch = 2, 5
    mp.start_processes(_rank_main, args=(world, _free_port(), global_batch, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    doc = shard.read_manifest(str(tmp_path / "manifest.json"))
    assert [s["n_samples"] for s in doc["shards"]] == [3, 2]
    # a single process tracing the whole batch and slicing per shard gives the same digests
    model = zoo.lenet5(batch=1)
    full = _ordered_records(model, graph_ref.calibrate(model.mod, model.params,
                                                       {"data": model.sample_inputs(0, global_batch)}, threads=1))
    for s in doc["shards"]:
        o, n = s["sample_offset"], s["n_samples"]
        sl = {k: v[o:o + n] for k, v in full.items()}
        assert shard.hex64(tf.records_digest(sl)) == s["digest"], s
    json.dumps(doc)

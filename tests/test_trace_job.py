"""Resumable trace generation (tachikoma_amd/trace_job.py; SURVEY.md §5 checkpoint/resume).

Host logic only: the chunk files here are written by a CPU tracer (the oracle's per-op
records through trace_format.trace_bytes), so a crash can be injected at any chunk and the
restarted job must trace exactly the missing chunks and end with the manifest an
uninterrupted job writes.  The device tracer (GraphModuleTracer) is covered by
tests/test_gpu_trace_job.py."""
import concurrent.futures
import json
import os

import numpy as np
import pytest

from tachikoma_amd import shard, trace_job, zoo
from tachikoma_amd import trace_format as tf


class CpuTracer:
    def __init__(self, fail_at=None):
        from oracle import graph_ref
        self.graph_ref = graph_ref
        self.model = zoo.lenet5(batch=1)
        self.calls = []
        self.fail_at = fail_at

    def __call__(self, offset, n, path):
        if self.fail_at is not None and len(self.calls) == self.fail_at:
            # a crash while the chunk's file is half written
            with open(path, "wb") as f:
                f.write(b"TKTRACE\0partial")
            raise RuntimeError("injected crash")
        self.calls.append(offset)
        x = self.model.sample_inputs(offset, n)
        recs = self.graph_ref.calibrate(self.model.mod, self.model.params, {"data": x}, threads=1)
        recs = {"data": recs["data"], **{k: v for k, v in recs.items() if k != "data"}}
        with open(path, "wb") as f:
            f.write(tf.trace_bytes({"sample_offset": offset, "n_samples": n}, {}, recs))
        fut = concurrent.futures.Future()
        fut.set_result(tf.records_digest(recs))
        return fut


def test_plan_chunks_tile_the_shard(tmp_path):
    for world in (1, 3):
        seen = []
        for r in range(world):
            cs = trace_job.plan_chunks(23, world, r, 4, str(tmp_path))
            assert [c.index for c in cs] == list(range(len(cs)))
            assert all(0 < c.n_samples <= 4 for c in cs)
            seen += [(c.sample_offset, c.n_samples) for c in cs]
        pos = 0
        for off, n in sorted(seen):
            assert off == pos
            pos += n
        assert pos == 23
    with pytest.raises(ValueError):
        trace_job.plan_chunks(8, 1, 0, 0, str(tmp_path))


def _manifest(tmp_path, entries, samples):
    p = str(tmp_path / "m.json")
    shard.write_manifest(p, "lenet5", samples, entries, world=1)
    return shard.read_manifest(p)


def test_crash_and_resume_traces_only_missing_chunks(tmp_path):
    ref_dir, run_dir = tmp_path / "ref", tmp_path / "run"
    full = trace_job.run(CpuTracer(), 11, 3, str(ref_dir))
    assert [e.n_samples for e in full] == [3, 3, 3, 2]

    crashing = CpuTracer(fail_at=2)
    with pytest.raises(RuntimeError):
        trace_job.run(crashing, 11, 3, str(run_dir))
    assert crashing.calls == [0, 3]
    assert len(trace_job.Journal(trace_job.journal_file(str(run_dir), 0)).entries()) == 2
    assert not os.path.exists(trace_job.chunk_file(str(run_dir), 0, 2))  # only the .partial exists

    resumed = CpuTracer()
    entries = trace_job.run(resumed, 11, 3, str(run_dir))
    assert resumed.calls == [6, 9]  # chunks 0 and 1 were kept
    assert [(e.sample_offset, e.n_samples, e.digest) for e in entries] == \
        [(e.sample_offset, e.n_samples, e.digest) for e in full]
    # the files hold the same records as the uninterrupted run's
    for e, f in zip(entries, full):
        assert tf.trace_file_digest(str(run_dir / e.file)) == int(f.digest, 16)
    doc = _manifest(tmp_path, entries, 11)
    assert [s["sample_offset"] for s in doc["shards"]] == [0, 3, 6, 9]

    # nothing left to do: a third run traces nothing
    again = CpuTracer()
    trace_job.run(again, 11, 3, str(run_dir))
    assert again.calls == []


def test_resume_redoes_damaged_chunks(tmp_path):
    d = str(tmp_path)
    trace_job.run(CpuTracer(), 8, 2, d)
    # chunk 1 truncated (size check), chunk 2 corrupted in place (digest check, verify only)
    c1 = trace_job.chunk_file(d, 0, 1)
    with open(c1, "rb+") as f:
        f.truncate(100)
    c2 = trace_job.chunk_file(d, 0, 2)
    raw = bytearray(open(c2, "rb").read())
    raw[-1] ^= 0xFF
    open(c2, "wb").write(bytes(raw))
    # a torn journal line from a crash during append is ignored
    with open(trace_job.journal_file(d, 0), "a") as f:
        f.write('{"chunk": 3, "sample_off')
    t = CpuTracer()
    trace_job.run(t, 8, 2, d)
    assert t.calls == [2]
    t = CpuTracer()
    entries = trace_job.run(t, 8, 2, d, verify=True)
    assert t.calls == [4]
    for e in entries:
        assert shard.hex64(tf.trace_file_digest(os.path.join(d, e.file))) == e.digest


def test_plan_change_is_not_resumed(tmp_path):
    d = str(tmp_path)
    trace_job.run(CpuTracer(), 6, 3, d)
    t = CpuTracer()
    trace_job.run(t, 6, 2, d)  # different chunking: every entry mismatches the plan
    assert t.calls == [0, 2, 4]
    t = CpuTracer()
    trace_job.run(t, 6, 2, d, resume=False)
    assert t.calls == [0, 2, 4]
    lines = open(trace_job.journal_file(d, 0)).read().strip().split("\n")
    assert len(lines) == 3 and all(json.loads(ln)["format"] == trace_job.JOURNAL_FORMAT for ln in lines)


def test_chunk_files_carry_sample_offsets(tmp_path):
    d = str(tmp_path)
    entries = trace_job.run(CpuTracer(), 5, 2, d, rank=1, world=2)
    off, n = shard.shard_range(5, 2, 1)
    assert entries[0].sample_offset == off and sum(e.n_samples for e in entries) == n
    tr = tf.read_trace(os.path.join(d, entries[0].file))
    assert tr.meta["sample_offset"] == off
    np.testing.assert_array_equal(tr.records["data"], zoo.lenet5(batch=1).sample_inputs(off, entries[0].n_samples))

"""Resumable trace generation on the MI355X (tachikoma_amd/trace_job.py): chunk files
produced by the device tracer (two pinned images, file written while the next chunk runs)
are bit-exact against the oracle, carry the device digest in the journal, and a job
interrupted after some chunks resumes with only the missing ones."""
import numpy as np
import pytest

from oracle import graph_ref
from tachikoma_amd import relay, shard, trace_job, zoo
from tachikoma_amd import trace_format as tf
from tachikoma_amd.contrib import graph_executor

pytestmark = pytest.mark.gpu


def _tracer(name):
    model_fn = zoo.MODELS[name]
    proto = model_fn(batch=1)

    def build_module(n):
        m = model_fn(batch=n)
        lib = relay.build(m.mod, target="mi355x", params=m.params)
        return graph_executor.GraphModule(lib["default"]())

    return proto, trace_job.GraphModuleTracer(build_module, proto.sample_inputs, model=proto.name,
                                              input_name=proto.input_name)


@pytest.mark.parametrize("name,samples,chunk", [("lenet5", 10, 4), ("resnet18", 6, 4)])
def test_device_trace_job_resume_bit_exact(device, tmp_path, name, samples, chunk):
    d = str(tmp_path)
    proto, tracer = _tracer(name)
    calls = []

    def crashing(offset, n, path):
        if len(calls) == 2:
            raise RuntimeError("injected crash")
        calls.append(offset)
        return tracer(offset, n, path)

    if samples > 2 * chunk:
        with pytest.raises(RuntimeError):
            trace_job.run(crashing, samples, chunk, d)
        assert len(trace_job.Journal(trace_job.journal_file(d, 0)).entries()) == 2
    resumed = []

    def counting(offset, n, path):
        resumed.append(offset)
        return tracer(offset, n, path)

    try:
        entries = trace_job.run(counting, samples, chunk, d, verify=True)
    finally:
        tracer.close()
    if samples > 2 * chunk:
        assert resumed == [2 * chunk]
    for e in entries:
        tr = tf.read_trace(f"{d}/{e.file}")
        assert tr.meta["sample_offset"] == e.sample_offset and tr.meta["n_samples"] == e.n_samples
        assert shard.hex64(tf.records_digest(tr.records)) == e.digest
        x = proto.sample_inputs(e.sample_offset, e.n_samples)
        exp = graph_ref.calibrate(proto.mod, proto.params, {proto.input_name: x}, backend="c")
        assert len(exp) == len(tr.records)
        for k, v in exp.items():
            assert np.array_equal(tr.records[k], v), (e.file, k)


def test_journal_digests_survive_a_slow_writer(device, tmp_path, monkeypatch):
    """Every chunk's journal digest is that chunk's own: the writer thread is slowed so the
    next same-size chunk's run (and digest) lands on the device before the value is read."""
    import time
    orig = graph_executor.TraceCapture.write

    def slow_write(self, path):
        time.sleep(0.3)
        orig(self, path)

    monkeypatch.setattr(graph_executor.TraceCapture, "write", slow_write)
    d = str(tmp_path)
    proto, tracer = _tracer("lenet5")
    try:
        entries = trace_job.run(tracer, 16, 4, d)
    finally:
        tracer.close()
    assert len(entries) == 4
    for e in entries:
        assert shard.hex64(tf.trace_file_digest(f"{d}/{e.file}")) == e.digest, e.file

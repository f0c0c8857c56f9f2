"""GraphModule boundary on the MI355X: traced runs never race with later writes, load_params
re-derives every build-time buffer, and a saved module reloads in a fresh process.

References: python/tvm/contrib/graph_executor.py:166-327 (set_input / run / load_params),
src/runtime/graph_executor/graph_executor.cc:283-291 (LoadParams), src/runtime/contrib/json/
json_runtime.h:105-135 (SaveToBinary / LoadFromBinary)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import graph_ref
from tachikoma_amd import _lib, relay, runtime, zoo
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.relay.build_module import lift_constants
from tachikoma_amd.trace_format import read_trace

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compare(records, expected):
    assert set(expected) <= set(records)
    for name, exp in expected.items():
        got = records[name]
        assert got.shape == exp.shape and got.dtype == exp.dtype, (name, got.shape, exp.shape)
        if not np.array_equal(got, exp):
            idx = tuple(np.argwhere(got != exp)[0])
            raise AssertionError(f"record {name}: first mismatch at {idx}: {got[idx]} vs {exp[idx]}")


def _image_records(m):
    return read_trace(m.trace_capture().bytes()).records


def test_traced_run_then_immediate_rewrite(device):
    """run(trace=True) returns while the D2H copies are in flight; an immediate set_input(B)
    and untraced run() must wait for them, so the image holds run A record for record."""
    import torch
    model = zoo.resnet18(batch=16)
    xa = model.sample_inputs(0, 16)
    xb = model.sample_inputs(16, 16)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input("data", xa)
    m.run(trace=True)
    m.set_input("data", xb)   # no synchronisation in between
    m.run()
    m.trace_capture().synchronize()
    torch.cuda.synchronize()
    recs = _image_records(m)
    exp = graph_ref.calibrate(model.mod, model.params, {"data": xa[[0, 15]]}, backend="c")
    _compare({k: v[[0, 15]] for k, v in recs.items()}, exp)
    # and the untraced run computed B
    out = m.get_output(0).numpy()
    exp_b = graph_ref.calibrate(model.mod, model.params, {"data": xb[[3]]}, backend="c")
    np.testing.assert_array_equal(out[[3]], exp_b[m.plan.outputs[0]])


def test_graph_replay_equals_plain_run(device):
    """tk_module_run_graph (one replayed HIP graph per run, the default) and tk_module_run give
    the same trace image byte for byte; the graph is re-used across runs with new inputs and a
    second pinned image (a second graph) holds its own run."""
    import torch
    model = zoo.lenet5(batch=8)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"]())
    xs = [model.sample_inputs(8 * i, 8) for i in range(3)]
    images = []
    for use_graph in (False, True):
        m.module.use_graph = use_graph
        for x in xs:
            m.set_input("data", x)
            m.run(trace=True)
            m.trace_capture().synchronize()
            images.append(bytes(m.trace_capture().bytes()))
    assert images[:3] == images[3:]
    assert images[0] != images[1]
    # copy kernels, memcpy nodes over 2 / 3 / 4 chains and 1 chain (the default packs the image)
    for mode in (1, 2, 3, 4, 5):
        _lib.check(m.module.lib.tk_module_set_graph_copies(m.module.handle, mode), "tk_module_set_graph_copies")
        m.set_input("data", xs[1])
        m.run(trace=True)
        m.trace_capture().synchronize()
        assert bytes(m.trace_capture().bytes()) == images[1], mode
    _lib.check(m.module.lib.tk_module_set_graph_copies(m.module.handle, 0), "tk_module_set_graph_copies")
    # packed capture with 1, 3 and more chunks than nodes; back-to-back runs (the two mirrors
    # alternate, kernels of run k+1 overlap the copies of run k)
    for chunks in (1, 3, 200, 8):
        _lib.check(m.module.lib.tk_module_set_trace_chunks(m.module.handle, chunks), "tk_module_set_trace_chunks")
        m.set_input("data", xs[2])
        for _ in range(3):
            m.run(trace=True)
        m.trace_capture().synchronize()
        assert bytes(m.trace_capture().bytes()) == images[2], chunks
    # a second image: its own graph; both images hold their own run
    cap2 = graph_executor.TraceCapture(m.module, m._meta)
    stream = torch.cuda.current_stream()
    m.set_input("data", xs[0])
    cap2.capture_inputs(stream)
    m.module.run(stream, cap2.capture_stream, cap2.host_dst)
    m.set_input("data", xs[2])
    m.run(trace=True)
    cap2.synchronize()
    m.trace_capture().synchronize()
    assert bytes(cap2.bytes()) == images[0]
    assert bytes(m.trace_capture().bytes()) == images[2]


def _reversed(params):
    """Same shapes, dtypes and value ranges, different values: each array reversed along axis 0."""
    return {k: np.ascontiguousarray(np.asarray(v)[::-1]) for k, v in params.items()}


@pytest.mark.parametrize("name,batch", [("resnet18", 2), ("qnn_dense_128", None), ("mobilenet_v2", 1)])
def test_load_params_repacks(device, tmp_path, name, batch):
    model = zoo.MODELS[name]() if batch is None else zoo.MODELS[name](batch=batch)
    x = model.fixed_input if batch is None else model.random_input()
    p2 = _reversed(model.params)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input(model.input_name, x)
    m.run(trace=True)                      # capture exists: its params section must refresh too
    m.load_params(relay.save_param_dict(p2))
    path = str(tmp_path / "p2.tkt")
    m.dump_trace(path)
    tr = read_trace(path)
    exp = graph_ref.calibrate(model.mod, p2, {model.input_name: x}, backend="c")
    _compare(tr.records, exp)
    for k, v in p2.items():
        np.testing.assert_array_equal(tr.params[k], v)


def test_load_params_realized_graph(device, tmp_path):
    """relay.quantize output: its folded weights are lifted to params (_const<k>) and the int8
    convolutions pack them; load_params re-packs."""
    from tachikoma_amd.relay.quantize import quantize
    fm = zoo.resnet_float(18, batch=2, hw=64)
    q = quantize(fm.mod, fm.params)
    mod_l, p1 = lift_constants(q, {})
    p2 = _reversed(p1)
    lib = relay.build(mod_l, target="mi355x", params=p1)
    m = graph_executor.GraphModule(lib["default"]())
    x = fm.random_input()
    m.set_input("data", x)
    m.load_params(relay.save_param_dict(p2))
    path = str(tmp_path / "q2.tkt")
    m.dump_trace(path)
    exp = graph_ref.calibrate(mod_l, p2, {"data": x})
    _compare(read_trace(path).records, exp)


def test_load_params_rejects_before_writing(device, tmp_path):
    model = zoo.resnet18(batch=1)
    x = model.random_input()
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input("data", x)
    bad = _reversed(model.params)
    first = next(iter(bad))
    bad[next(reversed(list(bad)))] = np.zeros((3, 3), np.int8)   # last entry has the wrong shape
    bad["not_in_graph"] = np.zeros(4, np.int32)                    # skipped like LoadParams
    with pytest.raises(_lib.TachikomaError):
        m.load_params(relay.save_param_dict(bad))
    # nothing was written: still the build-time params
    np.testing.assert_array_equal(m.get_input(first).numpy(), model.params[first])
    path = str(tmp_path / "p1.tkt")
    m.dump_trace(path)
    exp = graph_ref.calibrate(model.mod, model.params, {"data": x}, backend="c")
    _compare(read_trace(path).records, exp)


def test_export_library_reload_in_fresh_process(device, tmp_path):
    model = zoo.resnet18(batch=2)
    x = model.random_input()
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    mod_path = str(tmp_path / "resnet18.tkm")
    lib.export_library(mod_path)
    x_path = str(tmp_path / "x.npy")
    np.save(x_path, x)
    out = str(tmp_path / "reloaded.tkt")
    code = ("import sys, numpy as np; sys.path.insert(0, %r)\n"
            "from tachikoma_amd import runtime\n"
            "from tachikoma_amd.contrib import graph_executor\n"
            "lib = runtime.load_module(%r)\n"
            "m = graph_executor.GraphModule(lib['default']())\n"
            "m.set_input('data', np.load(%r))\n"
            "m.dump_trace(%r)\n") % (ROOT, mod_path, x_path, out)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    exp = graph_ref.calibrate(model.mod, model.params, {"data": x}, backend="c")
    _compare(read_trace(out).records, exp)


@pytest.mark.parametrize("mode", [0, 2, 4])
def test_graph_mode_small_modules(device, mode):
    """Graph runs of modules with 1-3 traced nodes (fewer than the copy chains): packed
    and memcpy-node captures give the host-issued run's image."""
    import numpy as np
    from tachikoma_amd.relay import qnn
    rng = np.random.default_rng(8)
    x = relay.var("x", (3, 40), "int32")
    e1 = qnn.op.requantize(x, relay.const(0.02), relay.const(1, "int32"), relay.const(0.5), relay.const(2, "int32"),
                           out_dtype="int8")
    e2 = relay.clip(e1, -20.0, 100.0)
    e3 = relay.cast(e2, "int32")
    for body in (e1, e2, e3):
        lib = relay.build(relay.IRModule.from_expr(body), target="mi355x", params={})
        m = graph_executor.GraphModule(lib["default"]())
        _lib.check(m.module.lib.tk_module_set_graph_copies(m.module.handle, mode), "tk_module_set_graph_copies")
        xv = rng.integers(-5000, 5000, (3, 40)).astype(np.int32)
        m.set_input("x", xv)
        m.module.use_graph = False
        m.run(trace=True)
        m.trace_capture().synchronize()
        want = bytes(m.trace_capture().bytes())
        m.module.use_graph = True
        for _ in range(2):
            m.run(trace=True)
        m.trace_capture().synchronize()
        assert bytes(m.trace_capture().bytes()) == want


def test_copy_trace_of_packed_runs(device):
    """tk_module_copy_trace: with tracing on, a packed traced run reports one entry per chunk copy
    whose bytes tile the mirrored image range, with ordered, non-overlapping copy intervals on the
    capture stream; the traced image is the same as without tracing; tracing off reports nothing new."""
    model = zoo.resnet18(batch=4)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"]())
    m.module.use_graph = True
    m.set_input("data", model.sample_inputs(0, 4))
    m.run(trace=True)
    m.trace_capture().synchronize()
    ref_img = bytes(m.trace_capture().bytes())
    m.module.set_copy_trace(True)
    for _ in range(2):
        m.run(trace=True)
        ch = m.module.copy_trace()
        assert 1 <= len(ch) <= 8  # the default 8 chunks (fewer where records complete late)
        assert all(c["bytes"] > 0 and c["end_ms"] >= c["start_ms"] >= 0 for c in ch)
        assert all(b["start_ms"] >= a["end_ms"] - 1e-3 for a, b in zip(ch, ch[1:]))
        # the chunks move the mirrored span of the op records (the graph inputs are copied by
        # capture_inputs; records the pack cannot move in whole 16-byte pieces go by their own copies)
        recs = sum(op.out.nbytes for op in m.plan.ops)
        assert 0.9 * recs <= sum(c["bytes"] for c in ch) <= m.trace_capture().layout.total
    m.trace_capture().synchronize()
    assert bytes(m.trace_capture().bytes()) == ref_img
    m.module.set_copy_trace(False)
    assert m.module.copy_trace() == []
    m.close()

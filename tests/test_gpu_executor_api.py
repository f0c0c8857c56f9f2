"""GraphModule / GraphModuleDebug device behaviour of the reference's remaining API names
(python/tvm/contrib/graph_executor.py:247-459, python/tvm/contrib/debugger/debug_executor.py:
252-503): share_params, benchmark, debug_get_output, run_individual(_node), profile."""
import numpy as np
import pytest

import tachikoma_amd
from oracle import graph_ref
from tachikoma_amd import relay, runtime, zoo
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.contrib.debugger import debug_executor

pytestmark = pytest.mark.gpu


def test_share_params_takes_the_other_modules_weights(device):
    """Two modules of one graph; the second gets different weights, then shares the first's: its
    output equals the first's (and the oracle's), so the packed MFMA weights were re-derived."""
    model = zoo.lenet5(batch=2)
    x = model.random_input()
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    a = graph_executor.GraphModule(lib["default"]())
    b = graph_executor.GraphModule(lib["default"]())
    rng = np.random.default_rng(3)
    other = {k: rng.integers(-128, 128, size=v.shape).astype(v.dtype) if v.dtype == np.int8 else v
             for k, v in model.params.items()}
    b.load_params(runtime.save_param_dict(other))
    for m in (a, b):
        m.set_input("data", x)
        m.run()
    assert not np.array_equal(a.get_output(0).numpy(), b.get_output(0).numpy())
    b.share_params(a, runtime.save_param_dict(model.params))
    b.run()
    exp = graph_ref.calibrate(model.mod, model.params, {"data": x})
    np.testing.assert_array_equal(b.get_output(0).numpy(), exp[b.plan.outputs[0]])
    np.testing.assert_array_equal(b.get_output(0).numpy(), a.get_output(0).numpy())


def test_benchmark(device):
    model = zoo.resnet18(batch=2)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = graph_executor.GraphModule(lib["default"](tachikoma_amd.rocm(0)))
    r = m.benchmark(tachikoma_amd.rocm(0), repeat=3, number=2, data=model.random_input())
    assert len(r.results) == 3 and 0 < r.min <= r.median <= r.max < 1.0
    r2 = m.benchmark(tachikoma_amd.rocm(0), repeat=2, number=1, end_to_end=True, data=model.random_input())
    assert len(r2.results) == 2 and r2.min > 0
    r3 = m.benchmark(tachikoma_amd.rocm(0), repeat=1, number=1, min_repeat_ms=20)
    assert len(r3.results) == 1 and r3.results[0] > 0


def test_debug_individual_timing_and_outputs(device, tmp_path):
    """run_individual: one list of `repeat` seconds per graph node, zeros for param nodes, positive
    for every fused node, and its per-node sum close to the whole-graph HIP-event node times;
    run_individual_node agrees; debug_get_output returns the oracle's value by index and name."""
    model = zoo.resnet18(batch=2)
    x = model.random_input()
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    m = debug_executor.create(lib, tachikoma_amd.rocm(0), dump_root=str(tmp_path / "dbg"))
    m.set_input("data", x)
    res = m.run_individual(number=5, repeat=2)
    nodes = m._nodes
    assert len(res) == len(nodes) and all(len(r) == 2 for r in res)
    for node, r in zip(nodes, res):
        if node["op"] == "param":
            assert r == [0.0, 0.0]
        else:
            assert all(0 < t < 0.1 for t in r), (node["name"], r)
    indiv = sum(min(r) for r in res)
    whole = sum(min(t) for t in m._node_times(3))
    assert 0.3 * whole < indiv < 3.0 * whole, (indiv, whole)
    big = max(range(len(res)), key=lambda i: min(res[i]))
    one = m.run_individual_node(big, number=5, repeat=3)
    assert len(one.results) == 3 and 0.3 * min(res[big]) < one.median < 3.0 * min(res[big])
    exp = graph_ref.calibrate(model.mod, model.params, {"data": x}, backend="c")
    outs = m.node_outputs()
    i = next(k for k, n in enumerate(nodes) if n["op"] != "param")
    np.testing.assert_array_equal(m.debug_get_output(i).numpy(), exp[outs[i]])
    buf = np.empty(exp[outs[big]].shape, exp[outs[big]].dtype)
    m.debug_get_output(nodes[big]["name"], buf)
    np.testing.assert_array_equal(buf, exp[outs[big]])
    with pytest.raises(AttributeError):
        m.debug_get_output("no-such-node")
    rep = m.profile(data=x)
    assert len(rep.calls) == sum(1 for n in nodes if n["op"] != "param")
    assert rep.configuration["Duration (us)"] > 0 and "Sum" in rep.table()
    m.exit()

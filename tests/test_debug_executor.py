"""Debug-executor dump: the reference's on-disk layout
(python/tvm/contrib/debugger/debug_result.py; checks mirror
tests/python/unittest/test_runtime_graph_debug.py:105-191)."""
import json
import os
import re

import numpy as np
import pytest

from tachikoma_amd import zoo
from tachikoma_amd.contrib.debugger.debug_executor import _debug_nodes, executor_graph_json
from tachikoma_amd.relay.build_module import lower


def test_executor_graph_json_layout():
    m = zoo.lenet5(batch=1)
    plan = lower(m.mod, m.params)
    g = executor_graph_json(plan)
    for k in ("nodes", "arg_nodes", "node_row_ptr", "heads", "attrs"):
        assert k in g
    n_args = len(plan.inputs) + len(plan.params)
    assert len(g["nodes"]) == n_args + len(plan.ops)
    assert g["arg_nodes"] == list(range(n_args))
    assert all(g["nodes"][i]["op"] == "null" for i in g["arg_nodes"])
    for i, node in enumerate(g["nodes"][n_args:], start=n_args):
        assert node["op"] == "tvm_op"
        assert all(src[0] < i for src in node["inputs"])  # topological
    assert g["node_row_ptr"] == list(range(len(g["nodes"]) + 1))
    assert len(g["attrs"]["dltype"][1]) == len(g["attrs"]["shape"][1]) == len(g["nodes"])
    nodes = _debug_nodes(g)
    assert nodes[0]["op"] == "param" and nodes[-1]["op"].startswith("tachikoma_")
    assert nodes[-1]["attrs"]["T"].startswith("type: ")


def test_fused_graph_json_layout():
    """granularity="fused": one tvm_op node per FuseOps group, named like the reference's
    fused functions, params as null nodes before their first consumer."""
    m = zoo.resnet18(batch=1)
    plan = lower(m.mod, m.params)
    g = executor_graph_json(plan, "fused")
    outputs = g.pop("outputs")
    ops = [n for n in g["nodes"] if n["op"] == "tvm_op"]
    from tachikoma_amd.relay.fuse import fused_nodes
    fns = fused_nodes(plan)
    assert [n["name"] for n in ops] == [f.node_name for f in fns]
    assert all(n["attrs"]["func_name"].startswith("tvmgen_default_fused_qnn_") or
               n["attrs"]["func_name"].startswith("tvmgen_default_fused_nn_") for n in ops)
    assert len(g["nodes"]) == len(plan.inputs) + len(plan.params) + len(fns)
    for i, n in enumerate(g["nodes"]):
        assert all(src[0] < i for src in n["inputs"])
    assert g["nodes"][g["heads"][0][0]]["op"] == "tvm_op"
    assert outputs[g["heads"][0][0]] == plan.outputs[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch", [("resnet18", 2), ("mobilenet_v2", 1)])
def test_fused_debug_dump_matches_oracle(device, tmp_path, name, batch):
    """Every fused node's dumped tensor equals the oracle's value of its group's last op."""
    import tachikoma_amd
    from oracle import graph_ref
    from tachikoma_amd import relay, trace_format as tf
    from tachikoma_amd.contrib.debugger import debug_executor

    model = zoo.MODELS[name](batch=batch)
    x = model.random_input()
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    mod = debug_executor.create(lib, tachikoma_amd.rocm(0), dump_root=str(tmp_path / "dbg"))
    mod.set_input("data", x)
    mod.run()
    with open(os.path.join(mod.dump_path, "output_tensors.params"), "rb") as f:
        tensors = tf.parse_ndarray_list(f.read(), copy=True)
    exp = graph_ref.calibrate(model.mod, model.params, {"data": x}, backend="c")
    pattern = re.compile(r"^(.+)____topo-index:(\d+)____output-num:0$")
    outs = mod.node_outputs()
    n_fused = 0
    for i, (key, arr) in enumerate(tensors.items()):
        mt = pattern.match(key)
        assert mt and int(mt.group(2)) == i
        src = outs[i]
        want = exp[src] if src in exp else model.params[src]
        np.testing.assert_array_equal(arr, want)
        n_fused += mt.group(1).startswith("tvmgen_default_fused_")
    from tachikoma_amd.relay.fuse import fused_nodes
    assert n_fused == len(fused_nodes(mod.plan))
    lines = mod.get_debug_result().split("\n")
    assert lines[-1].startswith("Total_time")
    mod.exit()


@pytest.mark.gpu
def test_debug_dump_matches_oracle(device, tmp_path):
    import tachikoma_amd
    from oracle import graph_ref
    from tachikoma_amd import relay, trace_format as tf
    from tachikoma_amd.contrib.debugger import debug_executor

    model = zoo.lenet5(batch=2)
    x = model.sample_inputs(0, 2)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    mod = debug_executor.create(lib, tachikoma_amd.rocm(0), dump_root=str(tmp_path / "dbg"), granularity="op")
    mod.set_input("data", x)
    directory = mod.dump_path
    assert os.path.basename(directory) == "_tvmdbg_device_ROCM_0"
    assert os.listdir(directory) == ["_tvmdbg_graph_dump.json"]
    with open(os.path.join(directory, "_tvmdbg_graph_dump.json")) as f:
        dumped = json.load(f)
    for k in ("nodes", "arg_nodes", "node_row_ptr", "heads", "attrs"):
        assert k in dumped
    mod.run()
    assert len(os.listdir(directory)) == 3

    with open(os.path.join(directory, "output_tensors.params"), "rb") as f:
        tensors = tf.parse_ndarray_list(f.read(), copy=True)
    exp = graph_ref.calibrate(model.mod, model.params, {"data": x})
    pattern = re.compile(r"^(.+)____topo-index:(\d+)____output-num:0$")
    seen = 0
    for i, (key, arr) in enumerate(tensors.items()):
        mt = pattern.match(key)
        assert mt and int(mt.group(2)) == i
        name = mt.group(1)
        want = exp[name] if name in exp else model.params[name]
        np.testing.assert_array_equal(arr, want)
        seen += 1
    assert seen == len(dumped["nodes"])

    with open(os.path.join(directory, "_tvmdbg_execution_trace.json")) as f:
        trace = json.load(f)
    assert trace["displayTimeUnit"] == "ns"
    events = trace["traceEvents"]
    assert len(events) == 2 * len(dumped["nodes"])
    assert all(e["ph"] in ("B", "E") and e["pid"] == 1 and e["tid"] == 1 for e in events)
    assert events[0]["ts"] == 0 and events[0]["ph"] == "B"

    lines = mod.get_debug_result().split("\n")
    assert re.split(r"  [ ]*", lines[0])[:-1] == ["Node Name", "Ops", "Time(us)", "Time(%)", "Shape", "Inputs",
                                                   "Outputs", "Measurements(us)"]
    assert lines[-1].startswith("Total_time")
    mod.exit()
    assert not os.path.exists(directory)


def test_canonical_graph_json_layout():
    """granularity="canonical": the fused functions of the canonicalized graph, with the
    reference's names (cast_subtract operand shifts, nn_conv2d_add_fixed_point_multiply_* blocks)."""
    from tachikoma_amd.relay.canonical import canonicalize
    from tachikoma_amd.relay.fuse import fused_nodes
    m = zoo.resnet18(batch=1)
    plan = lower(m.mod, m.params)
    g = executor_graph_json(plan, "canonical")
    outputs = g.pop("outputs")
    ops = [n for n in g["nodes"] if n["op"] == "tvm_op"]
    fns = fused_nodes(canonicalize(plan))
    assert [n["name"] for n in ops] == [f.node_name for f in fns]
    names = {n["attrs"]["func_name"] for n in ops}
    assert any(f.startswith("tvmgen_default_fused_cast_subtract") for f in names)
    assert any(f.startswith("tvmgen_default_fused_nn_conv2d_add_fixed_point_multiply_per_axis") for f in names)
    assert not any("qnn_" in f for f in names)
    for i, n in enumerate(g["nodes"]):
        assert all(src[0] < i for src in n["inputs"])
    assert len(outputs) == len(g["nodes"])


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch", [("resnet18", 2), ("mobilenet_v2", 1), ("lenet5_tonearest", 2)])
def test_canonical_debug_dump_matches_oracle(device, tmp_path, name, batch):
    """Every canonical fused node's dumped tensor -- plan records and the device-computed
    intermediates (int16 operand shifts, int32 partial requantize / add results) -- equals the
    CPU evaluation of the canonical ops (oracle/canonical_ref.py)."""
    import tachikoma_amd
    from oracle import canonical_ref
    from tachikoma_amd import relay, trace_format as tf
    from tachikoma_amd.contrib.debugger import debug_executor

    if name.endswith("_tonearest"):
        from tachikoma_amd.relay import qnn
        with qnn.op.requantize_config(rounding="TONEAREST"):
            model = zoo.MODELS[name.rsplit("_", 1)[0]](batch=batch)
    else:
        model = zoo.MODELS[name](batch=batch)
    x = model.random_input()
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    mod = debug_executor.create(lib, tachikoma_amd.rocm(0), dump_root=str(tmp_path / "dbg"), granularity="canonical")
    mod.set_input("data", x)
    mod.run()
    with open(os.path.join(mod.dump_path, "output_tensors.params"), "rb") as f:
        tensors = tf.parse_ndarray_list(f.read(), copy=True)
    exp = canonical_ref.evaluate(mod.canon, {"data": x, **{k: np.asarray(v) for k, v in model.params.items()}})
    pattern = re.compile(r"^(.+)____topo-index:(\d+)____output-num:0$")
    outs = mod.node_outputs()
    computed = 0
    ops = {o.name: o for o in mod.canon.ops}
    for i, (key, arr) in enumerate(tensors.items()):
        mt = pattern.match(key)
        assert mt and int(mt.group(2)) == i
        np.testing.assert_array_equal(arr, exp[outs[i]], err_msg=key)
        computed += outs[i] in ops and ops[outs[i]].record is None
    assert computed > 0  # the int16 shifts at least were evaluated on the device
    assert mod.get_debug_result().split("\n")[-1].startswith("Total_time")
    mod.exit()

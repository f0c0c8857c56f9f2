"""The GraphModule / GraphModuleDebug Python surface against the reference's names, argument
lists and return shapes (python/tvm/contrib/graph_executor.py:247-459,
python/tvm/contrib/debugger/debug_executor.py:252-503), on the CPU: signatures, the host-side
logic that needs no device, and the BenchmarkResult / Report containers.  The device behaviour is
tests/test_gpu_executor_api.py."""
import inspect
import json

import numpy as np
import pytest

from tachikoma_amd import zoo
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.contrib.debugger import debug_executor
from tachikoma_amd.relay.build_module import lower


class _Stub:
    """The part of a DeviceModule GraphModule.__init__ reads (no device)."""

    def __init__(self, plan):
        self.plan = plan


@pytest.fixture(scope="module")
def lenet_module():
    m = zoo.lenet5(batch=1)
    return graph_executor.GraphModule(_Stub(lower(m.mod, m.params)))


def _params(fn):
    return [(p.name, p.default) for p in inspect.signature(fn).parameters.values()]


def test_graph_module_signatures():
    G = graph_executor.GraphModule
    assert _params(G.get_input_index) == [("self", inspect._empty), ("name", inspect._empty)]
    assert _params(G.share_params) == [("self", inspect._empty), ("other", inspect._empty),
                                       ("params_bytes", inspect._empty)]
    assert [n for n, _ in _params(G.debug_get_output)] == ["self", "node", "out"]
    bench = dict(_params(G.benchmark))
    assert bench["func_name"] == "run" and bench["repeat"] == 5 and bench["number"] == 5
    assert bench["min_repeat_ms"] is None and bench["limit_zero_time_iterations"] == 100
    assert bench["end_to_end"] is False and bench["cooldown_interval_ms"] == 0 and bench["repeats_to_cooldown"] == 1


def test_debug_module_signatures():
    D = debug_executor.GraphModuleDebug
    ri = dict(_params(D.run_individual))
    assert list(ri)[:2] == ["self", "number"] and ri["number"] is inspect._empty
    assert ri["repeat"] == 1 and ri["min_repeat_ms"] == 0 and ri["limit_zero_time_iterations"] == 100
    rin = dict(_params(D.run_individual_node))
    assert list(rin)[:2] == ["self", "index"] and rin["number"] == 10 and rin["repeat"] == 1
    assert [n for n, _ in _params(D.debug_get_output)] == ["self", "node", "out"]
    assert [n for n, _ in _params(D.profile)][:2] == ["self", "collectors"]


def test_input_index_and_info(lenet_module):
    m = lenet_module
    assert m.get_input_index("data") == 0
    assert m.get_input_index("nope") == -1
    shapes, dtypes = m.get_input_info()
    assert shapes == {"data": (1, 1, 28, 28)} and dtypes == {"data": "int8"}
    # weights are params, not inputs (graph_executor.py:264-272)
    assert all(not k.startswith("w") for k in shapes)


def test_getitem_and_plain_debug_get_output(lenet_module):
    m = lenet_module
    assert m["get_input_index"]("data") == 0
    assert m["get_num_inputs"]() == 1
    with pytest.raises(AttributeError):
        m["no_such_function"]
    with pytest.raises(NotImplementedError, match="debug_executor"):
        m.debug_get_output(0, None)


def test_trace_header_names_the_compute_dtype():
    from tachikoma_amd.relay import qnn
    m = zoo.lenet5(batch=1)
    assert graph_executor._compute_dtypes(lower(m.mod, m.params)) == "int64"
    with qnn.op.requantize_config(compute_dtype="float64"):
        m = zoo.lenet5(batch=1)
    assert graph_executor._compute_dtypes(lower(m.mod, m.params)) == "float64"


def test_benchmark_result_statistics():
    r = graph_executor.BenchmarkResult([0.003, 0.001, 0.002])
    assert r.min == 0.001 and r.max == 0.003 and r.median == 0.002
    assert abs(r.mean - 0.002) < 1e-15 and abs(r.std - np.std([0.003, 0.001, 0.002])) < 1e-15
    assert "mean (ms)" in str(r) and "BenchmarkResult(" in repr(r)


def test_report_renderings():
    calls = [{"Name": "a", "Duration (us)": 30.0, "Percent": 75.0, "Count": 1, "Device": "rocm0", "Hash": "x",
              "Argument Shapes": "(1,)"},
             {"Name": "b", "Duration (us)": 10.0, "Percent": 25.0, "Count": 1, "Device": "rocm0", "Hash": "y",
              "Argument Shapes": "(2,)"}]
    rep = debug_executor.Report(calls, {"Executor": "GraphModuleDebug"})
    lines = rep.table().split("\n")
    assert lines[0].split()[0] == "Name" and lines[1].startswith("a") and lines[3].startswith("Sum")
    assert json.loads(rep.json())["calls"][1]["Name"] == "b"
    assert rep.csv().split("\n")[0].startswith('"Name"')

"""Relay graph ingestion through the device: a graph saved as Relay
text (``IRModule.astext``) plus a params blob written by ``save_param_dict`` (the reference's
``SaveParams`` NDArray-list, src/runtime/file_utils.cc:184-206) is read back from files,
parsed (``tvm.parser.parse``), built with ``relay.build(mod, params=<bytes>)``
(python/tvm/relay/build_module.py:409) and traced on the MI355X; every record must equal the
oracle's record of the constructor-built graph."""
import numpy as np
import pytest

from oracle import graph_ref
from tachikoma_amd import relay, zoo
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.trace_format import read_trace

pytestmark = pytest.mark.gpu


def _save_and_reload(mod, params, tmp_path):
    text_path, params_path = tmp_path / "graph.relay", tmp_path / "graph.params"
    text_path.write_text(mod.astext())
    params_path.write_bytes(relay.save_param_dict(params))
    return relay.parse(text_path.read_text()), params_path.read_bytes()


def _trace_records(mod, blob, input_name, x, tmp_path):
    lib = relay.build(mod, target="mi355x", params=blob)
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input(input_name, x)
    path = str(tmp_path / "parsed.tkt")
    m.dump_trace(path)
    return read_trace(path).records


def _compare(records, expected):
    assert len(records) == len(expected)
    for name, exp in expected.items():
        got = records[name]
        assert got.shape == exp.shape and got.dtype == exp.dtype, name
        if not np.array_equal(got, exp):
            idx = tuple(np.argwhere(got != exp)[0])
            raise AssertionError(f"record {name}: first mismatch at {idx}: {got[idx]} vs {exp[idx]}")


@pytest.mark.parametrize("name,batch", [("resnet18", 2), ("mobilenet_v2", 1), ("lenet5", 4)])
def test_parsed_text_and_params_file_trace(device, tmp_path, name, batch):
    model = zoo.MODELS[name](batch=batch)
    x = model.random_input()
    mod, blob = _save_and_reload(model.mod, model.params, tmp_path)
    records = _trace_records(mod, blob, model.input_name, x, tmp_path)
    exp = graph_ref.calibrate(model.mod, model.params, {model.input_name: x}, backend="c")
    _compare(records, exp)


def test_parsed_realized_graph_trace(device, tmp_path):
    """A relay.quantize-realized graph (float32 input quantize, int8 nn.conv2d, shifts,
    fixed_point_multiply, float32 classifier) through text and a params file."""
    from tachikoma_amd.relay.build_module import lift_constants
    from tachikoma_amd.relay.quantize import quantize
    fm = zoo.resnet_float(18, batch=2, hw=32)
    q = quantize(fm.mod, fm.params)
    lifted, params = lift_constants(q, {})
    mod, blob = _save_and_reload(lifted, params, tmp_path)
    x = fm.random_input()
    records = _trace_records(mod, blob, "data", x, tmp_path)
    exp = graph_ref.calibrate(q, {}, {"data": x})
    assert set(exp) <= set(records)
    for name in list(records):
        if name not in exp:
            records.pop(name)
    _compare(records, exp)


@pytest.mark.parametrize("name", ["mnist", "mobilenet", "resnet50"])
def test_reference_relay_text_quantized_trace(device, tmp_path, name):
    """The reference's own float models as Relay text (tests/python/relay/collage/menangerie.py,
    extracted to tests/golden/menangerie_*.relay; batch norms, explicit padding), parsed,
    quantized (SimplifyInference / FoldScaleAxis folding the batch norms first), built and traced
    on the MI355X: every record bit-exact against the oracle run of the same quantized graph."""
    from tachikoma_amd.relay.quantize import quantize
    from .golden_util import menangerie
    mod, iname, shape = menangerie(name)
    q = quantize(mod, {})
    x = np.random.default_rng(7).standard_normal(shape).astype(np.float32)
    lib = relay.build(q, target="mi355x")
    m = graph_executor.GraphModule(lib["default"]())
    m.set_input(iname, x)
    path = str(tmp_path / f"{name}.tkt")
    m.dump_trace(path)
    records = read_trace(path).records
    exp = graph_ref.calibrate(q, {}, {iname: x})
    assert set(exp) <= set(records)
    for k, v in exp.items():
        got = records[k]
        assert got.shape == v.shape and got.dtype == v.dtype, k
        if not np.array_equal(got, v):
            idx = tuple(np.argwhere(got != v)[0])
            raise AssertionError(f"{name} record {k}: first mismatch at {idx}: {got[idx]} vs {v[idx]}")

"""Host side of module serialisation and build hygiene (no GPU needed).

* save_param_dict / load_param_dict round trip (python/tvm/runtime/params.py:22-69);
* export_library → load_module reproduces the lowered plan exactly (SaveToBinary /
  LoadFromBinary, src/runtime/contrib/json/json_runtime.h:105-135);
* build(params=<blob>) accepts a params blob like relay.build(..., params) after
  load_param_dict (python/tvm/relay/build_module.py:409);
* the library carries the digest of the sources it was built from, and the loader refuses
  a stale one."""
import ctypes
import json

import numpy as np
import pytest

from tachikoma_amd import _lib, relay, runtime, zoo
from tachikoma_amd import build as tkbuild
from tachikoma_amd.relay.build_module import lift_constants


def test_param_dict_round_trip():
    rng = np.random.default_rng(0)
    params = {"w": rng.integers(-128, 128, (4, 3, 3, 3), dtype=np.int8),
              "b": rng.integers(-1000, 1000, (4,), dtype=np.int32),
              "f": rng.standard_normal((2, 5)).astype(np.float32)}
    blob = relay.save_param_dict(params)
    back = relay.load_param_dict(blob)
    assert list(back) == list(params)
    for k in params:
        assert back[k].dtype == params[k].dtype
        np.testing.assert_array_equal(back[k], params[k])


def _plans_equal(a, b):
    assert runtime.plan_to_json(a) == runtime.plan_to_json(b)
    for oa, ob in zip(a.ops, b.ops):
        assert set(oa.consts) == set(ob.consts)
        for k in oa.consts:
            assert oa.consts[k].dtype == ob.consts[k].dtype
            np.testing.assert_array_equal(oa.consts[k], ob.consts[k])


@pytest.mark.parametrize("name", ["qnn_dense_128", "lenet5", "resnet18", "mobilenet_v2"])
def test_export_library_round_trip(tmp_path, name):
    model = zoo.MODELS[name]()
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    path = str(tmp_path / f"{name}.tkm")
    lib.export_library(path)
    back = runtime.load_module(path)
    _plans_equal(lib.plan, back.plan)
    assert back.fuse == lib.fuse and back.target == lib.target and back.mod_name == lib.mod_name
    for k, v in lib.params.items():
        assert back.params[k].dtype == v.dtype
        np.testing.assert_array_equal(back.params[k], v)
    # the graph json is the plan
    assert json.loads(lib.get_graph_json()) == runtime.plan_to_json(back.plan)


def test_export_library_realized_graph(tmp_path):
    """A relay.quantize result: lifted constants, float attrs (realized scales), per-channel
    requantize constants all survive."""
    from tachikoma_amd.relay.quantize import quantize
    fm = zoo.resnet_float(18, batch=1, hw=32)
    q = quantize(fm.mod, fm.params)
    lib = relay.build(q, target="mi355x")
    back = runtime.deserialize_module(lib.save())
    _plans_equal(lib.plan, back.plan)


def test_module_rejects_corrupt_files():
    model = zoo.qnn_dense_128()
    data = relay.build(model.mod, target="mi355x", params=model.params).save()
    with pytest.raises(ValueError):
        runtime.deserialize_module(b"XXXXXXXX" + data[8:])
    with pytest.raises(ValueError):
        runtime.deserialize_module(data[:100])


def test_build_accepts_params_blob():
    model = zoo.lenet5()
    blob = relay.save_param_dict(model.params)
    a = relay.build(model.mod, target="mi355x", params=model.params)
    b = relay.build(model.mod, target="mi355x", params=blob)
    _plans_equal(a.plan, b.plan)
    for k in a.params:
        np.testing.assert_array_equal(a.params[k], b.params[k])


def test_lifted_params_round_trip_blob():
    """load_params input for a realized graph: the lifted constants as a blob."""
    from tachikoma_amd.relay.quantize import quantize
    fm = zoo.resnet_float(18, batch=1, hw=32)
    q = quantize(fm.mod, fm.params)
    _, params = lift_constants(q, {})
    assert params and all(k.startswith("_const") for k in params)
    back = relay.load_param_dict(relay.save_param_dict(params))
    for k, v in params.items():
        np.testing.assert_array_equal(back[k], v)


def test_library_carries_source_digest():
    lib = _lib.load()
    assert lib.tk_build_info().decode().split("+")[0] == tkbuild.source_hash()
    assert _lib.build_info() == tkbuild.source_hash()


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A library built from other sources must not load (a stale .so pushed to a GPU box)."""
    monkeypatch.setattr(tkbuild, "source_hash", lambda: "0000000000000000")
    monkeypatch.setattr(_lib, "_LIB", None)
    with pytest.raises(_lib.TachikomaError, match="other sources"):
        _lib.load()
    monkeypatch.undo()
    _lib._LIB = None
    _lib.load()


def test_product_library_ignores_tuning_env(monkeypatch):
    """Kernel-selection switches are compiled out of the product build: the ablation-only
    variables leave the scratch plan (which depends on the split-K / wide-stage choice)
    unchanged."""
    from tachikoma_amd._lib import TensorRef, tk_conv2d_attrs
    lib = _lib.load()
    x = TensorRef(0, (16, 2048, 7, 7), "int8")
    w = TensorRef(0, (512, 2048, 1, 1), "int8")
    a = tk_conv2d_attrs()
    a.strides[:] = [1, 1]
    a.dilation[:] = [1, 1]
    a.groups = 1
    base = lib.tk_conv2d_scratch_bytes(x.ptr, w.ptr, ctypes.byref(a), 1)
    assert base > 0  # this shape takes split-K partial tiles
    for k, v in {"TK_WIDE": "0", "TK_WIDE_MAX_TILES": "0", "TK_RING": "5", "TK_MT2": "1", "TK_IMGTILE": "0"}.items():
        monkeypatch.setenv(k, v)
    assert lib.tk_conv2d_scratch_bytes(x.ptr, w.ptr, ctypes.byref(a), 1) == base

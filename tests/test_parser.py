"""Relay text ingestion: tvm.parser.parse / IRModule.astext for the
integer QNN subset, including the #[metadata] section (src/node/serialization.cc layout)."""
import base64
import json
import struct

import numpy as np
import pytest

from oracle import graph_ref
from tachikoma_amd import relay, zoo
from tachikoma_amd.relay import parser
from tachikoma_amd.relay.build_module import lower


def _same_plan(m1, m2, params):
    p1, p2 = lower(m1, params), lower(m2, params)
    assert [o.name for o in p1.ops] == [o.name for o in p2.ops]
    for a, b in zip(p1.ops, p2.ops):
        assert a.op == b.op and a.inputs == b.inputs and a.attrs == b.attrs, a.name
        assert a.consts.keys() == b.consts.keys()
        for k in a.consts:
            np.testing.assert_array_equal(a.consts[k], b.consts[k])


@pytest.mark.parametrize("name", ["qnn_dense_128", "lenet5", "resnet18", "mobilenet_v2", "resnet50"])
def test_astext_parse_roundtrip(name):
    m = zoo.MODELS[name]() if name == "qnn_dense_128" else zoo.MODELS[name](batch=1)
    text = m.mod.astext()
    assert text.startswith('#[version = "0.0.5"]')
    _same_plan(m.mod, relay.parse(text), m.params)


def _dltensor_b64(a):
    a = np.ascontiguousarray(a)
    code = {"i": 0, "u": 1, "f": 2}[a.dtype.kind]
    blob = struct.pack("<QQiii", 0xDD5E40F096B4A13F, 0, 1, 0, a.ndim) + struct.pack("<BBH", code, a.itemsize * 8, 1)
    blob += struct.pack(f"<{a.ndim}q", *a.shape) + struct.pack("<q", a.nbytes) + a.tobytes()
    return base64.b64encode(blob).decode()


# written the way TVM 0.11's text printer emits it (type annotations, float32 'f' literals,
# metadata constants), with the metadata JSON built independently of parser.dump_meta_json
TVM_STYLE = '''#[version = "0.0.5"]
def @main(%x: Tensor[(2, 8, 6, 6), int8] /* ty=Tensor[(2, 8, 6, 6), int8] */, %w: Tensor[(16, 8, 3, 3), int8] /* ty=Tensor[(16, 8, 3, 3), int8] */, %b: Tensor[(16), int32] /* ty=Tensor[(16), int32] */) -> Tensor[(2, 16, 6, 6), int8] {
  %0 = qnn.conv2d(%x, %w, -3 /* ty=int32 */, 0 /* ty=int32 */, 0.05f /* ty=float32 */, meta[relay.Constant][0] /* ty=Tensor[(16), float32] */, padding=[1, 1, 1, 1], channels=16, kernel_size=[3, 3], out_dtype="int32") /* ty=Tensor[(2, 16, 6, 6), int32] */;
  %1 = nn.bias_add(%0, %b) /* ty=Tensor[(2, 16, 6, 6), int32] */;
  %2 = qnn.requantize(%1, meta[relay.Constant][1] /* ty=Tensor[(16), float32] */, 0 /* ty=int32 */, 0.25f /* ty=float32 */, 4 /* ty=int32 */, axis=1, out_dtype="int8") /* ty=Tensor[(2, 16, 6, 6), int8] */;
  // ReLU in the quantised domain
  clip(%2, a_min=4f, a_max=127f) /* ty=Tensor[(2, 16, 6, 6), int8] */
}

#[metadata]
'''


def test_parse_tvm_printed_text():
    rng = np.random.default_rng(0)
    s_w = rng.uniform(0.002, 0.02, 16).astype(np.float32)
    s_in = (np.float32(0.05) * s_w).astype(np.float32)
    meta = {"root": 1, "nodes": [{"type_key": ""}, {"type_key": "Map", "keys": ["relay.Constant"], "data": [2]},
                                 {"type_key": "Array", "data": [3, 4]},
                                 {"type_key": "relay.Constant", "attrs": {"data": "0", "span": "0"}},
                                 {"type_key": "relay.Constant", "attrs": {"data": "1", "span": "0"}}],
            "b64ndarrays": [_dltensor_b64(s_w), _dltensor_b64(s_in)], "attrs": {"tvm_version": "0.11.dev0"}}
    mod = relay.parse(TVM_STYLE + json.dumps(meta))
    # the same graph through the constructors
    x = relay.var("x", shape=(2, 8, 6, 6), dtype="int8")
    w = relay.var("w", shape=(16, 8, 3, 3), dtype="int8")
    b = relay.var("b", shape=(16,), dtype="int32")
    y = relay.qnn.op.conv2d(x, w, relay.const(-3, "int32"), relay.const(0, "int32"), relay.const(0.05, "float32"),
                            relay.const(s_w), kernel_size=(3, 3), channels=16, padding=(1, 1))
    y = relay.nn.bias_add(y, b)
    y = relay.qnn.op.requantize(y, relay.const(s_in), relay.const(0, "int32"), relay.const(0.25, "float32"),
                                relay.const(4, "int32"), axis=1, out_dtype="int8")
    y = relay.clip(y, 4.0, 127.0)
    ref_mod = relay.IRModule.from_expr(y)
    params = {"w": rng.integers(-128, 128, (16, 8, 3, 3)).astype(np.int8),
              "b": rng.integers(-1000, 1000, 16).astype(np.int32)}
    _same_plan(ref_mod, mod, params)
    xin = rng.integers(-128, 128, (2, 8, 6, 6)).astype(np.int8)
    r1 = graph_ref.calibrate(mod, params, {"x": xin})
    r2 = graph_ref.calibrate(ref_mod, params, {"x": xin})
    assert r1.keys() == r2.keys()
    for k in r1:
        np.testing.assert_array_equal(r1[k], r2[k])


def test_meta_json_roundtrip_and_literals():
    arrs = [np.arange(6, dtype=np.float32).reshape(2, 3), np.array([1, -2], np.int8), np.array(5, np.int64)]
    back = parser.load_meta_json(parser.dump_meta_json(arrs))["relay.Constant"]
    for a, b in zip(arrs, back):
        assert a.dtype == b.dtype
        np.testing.assert_array_equal(a, b)
    assert parser._number("3") == np.int32(3) and parser._number("3").dtype == np.int32
    assert parser._number("3i64").dtype == np.int64 and parser._number("2u8").dtype == np.uint8
    assert parser._number("0.5f").dtype == np.float32 and parser._number("1e-05f") == np.float32(1e-05)
    assert parser._number("2f64").dtype == np.float64


def test_parse_errors():
    with pytest.raises(relay.ParseError):
        relay.parse('def @main(%x: Tensor[(4), int8]) { nn.softmax(%x) }')
    with pytest.raises(relay.ParseError):
        relay.parse('def @main(%x: Tensor[(4), int8]) { cast(%y, dtype="int32") }')
    with pytest.raises(relay.ParseError):
        relay.parse('def @main(%x: Tensor[(4), int8]) { qnn.add(%x, %x, meta[relay.Constant][3], 0, 1f, 0, 1f, 0) }')


def test_parenthesised_expression_is_grouping_not_tuple():
    """`(%x)` groups (a tensor), `(%x,)` is a 1-tuple, `()` the empty tuple (Relay's text format)."""
    from tachikoma_amd.relay.expr import Tuple
    m = relay.parse('def @main(%x: Tensor[(4), int8]) { cast((%x), dtype="int32") }')
    assert m["main"].body.op == "cast" and not isinstance(m["main"].body.args[0], Tuple)
    m = relay.parse('def @main(%x: Tensor[(2, 3), int8]) { qnn.concatenate((%x,), (0.5f,), (0,), 0.5f, 0, axis=0) }')
    (tup,) = [a for a in m["main"].body.args[:1]]
    assert isinstance(tup, Tuple) and len(tup.fields) == 1

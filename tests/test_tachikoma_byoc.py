"""tachikoma BYOC composites (tachikoma.qnn.conv2d / tachikoma.qnn.dense), SURVEY.md §8(f) row 3.

Models are built the way the reference's tests build them (tests/python/contrib/
test_tachikoma.py:1422-1616 ``test_qnn_conv2d`` profiles, :1702-1762 ``test_qnn_dense``):
uint8 data in [0, 20], int8 weights in [-20, 20], int32 bias in [-50, 50], requantize to
int32 -> clip(0, 255) -> cast(uint8) [-> qnn.add(., sum_in uint8 [0, 10]) -> clip(0, 255)],
with the reference's quantization profiles.  Checks:
  * the partitioner's folded float32 constants equal oracle/tachikoma_ref.legalize_constants
    (an independent restatement of LegalizeQnnOpForTachikoma, tachikoma.py:1239-1253);
  * the composite result is within +-1 quantum of the QNN lowering — the reference test's own
    tolerance (test_tachikoma.py:1615-1616, 1761-1762);
  * on the GPU: the composite record is bit-exact against the oracle's post-op chain and the
    unpartitioned QNN graph is bit-exact against the QNN oracle.
"""
import numpy as np
import pytest

from oracle import graph_ref, tachikoma_ref
from tachikoma_amd import relay
from tachikoma_amd.relay.build_module import lower
from tachikoma_amd.relay.contrib import tachikoma as tkbyoc

# (d_zp, d_scl, k_scl, rq_zp, rq_scl, sum_zp, sum_scl, o_zp, o_scl): test_tachikoma.py:1485-1504
QP_REGULAR = (0, 0.2, 0.1, 30, 0.2, 15, 0.3, 5, 0.2)
QP_ASYM = (3, 0.2, 0.1, 10, 0.1, 15, 0.3, 4, 0.2)

# name: (shape NCHW, kernel, pad, groups, OC, bias, sum, quant profile): test_tachikoma.py:1436-1521
CONV_PROFILES = {
    "Base": ((1, 8, 5, 5), 3, 1, 1, 16, True, False, QP_REGULAR),
    "NoBias": ((1, 8, 5, 5), 3, 1, 1, 16, False, False, QP_REGULAR),
    "Group": ((1, 8, 5, 5), 3, 0, 2, 16, True, False, QP_ASYM),
    "DW": ((1, 16, 5, 5), 3, 0, 16, 16, True, False, QP_ASYM),
    "AsymmetricInput": ((1, 8, 5, 5), 3, 0, 1, 16, True, False, QP_ASYM),
    "WithSum": ((1, 8, 5, 5), 3, 0, 1, 16, True, True, QP_ASYM),
    "WithSum_NoBias": ((1, 8, 5, 5), 3, 0, 1, 16, False, True, QP_ASYM),
    # larger cases whose contraction takes the MFMA path on the GPU (an input zero point with
    # padding breaks the legalization at the borders, as the reference notes: test_tachikoma.py:1511)
    "MFMA": ((2, 64, 14, 14), 3, 0, 1, 64, True, True, QP_ASYM),
    "MFMA_Pad": ((2, 64, 14, 14), 3, 1, 1, 128, True, False, QP_REGULAR),
}
# name: (N, IC, OC, bias, sum, profile): test_tachikoma.py:1455-1456, 1702-1762
DENSE_PROFILES = {
    "Base": (2, 10, 16, True, False, QP_REGULAR),
    "NoBias": (2, 10, 16, False, False, QP_REGULAR),
    "WithSum": (2, 10, 16, True, True, QP_ASYM),
    "Big": (64, 256, 128, True, True, QP_ASYM),
}


def _qnn_tail(op, q, out_shape, with_sum, rng, params, inputs):
    d_zp, d_scl, k_scl, rq_zp, rq_scl, sum_zp, sum_scl, o_zp, o_scl = q
    rq_in_scl = np.float32(np.float32(d_scl) * np.float32(k_scl))
    op = relay.qnn.op.requantize(op, relay.const(rq_in_scl), relay.const(0), relay.const(np.float32(rq_scl)),
                                 relay.const(rq_zp), out_dtype="int32")
    op = relay.clip(op, 0.0, 255.0)
    op = relay.cast(op, "uint8")
    if with_sum:
        inputs["sum_in"] = rng.integers(0, 11, size=out_shape).astype(np.uint8)
        s = relay.var("sum_in", shape=out_shape, dtype="uint8")
        op = relay.qnn.op.add(op, s, relay.const(np.float32(rq_scl)), relay.const(rq_zp),
                              relay.const(np.float32(sum_scl)), relay.const(sum_zp),
                              relay.const(np.float32(o_scl)), relay.const(o_zp))
        op = relay.clip(op, 0.0, 255.0)
    return op


def conv_model(name):
    shape, k, pad, groups, oc, bias, with_sum, q = CONV_PROFILES[name]
    rng = np.random.default_rng(0)
    n, c, h, w = shape
    d_zp, d_scl, k_scl = q[0], q[1], q[2]
    params, inputs = {}, {"data": rng.integers(0, 21, size=shape).astype(np.uint8)}
    params["weight"] = rng.integers(-20, 21, size=(oc, c // groups, k, k)).astype(np.int8)
    data = relay.var("data", shape=shape, dtype="uint8")
    wgt = relay.var("weight", shape=params["weight"].shape, dtype="int8")
    op = relay.qnn.op.conv2d(data, wgt, relay.const(d_zp), relay.const(0), relay.const(np.float32(d_scl)),
                             relay.const(np.float32(k_scl)), kernel_size=(k, k), channels=oc, padding=(pad, pad),
                             groups=groups)
    if bias:
        params["bias"] = rng.integers(-50, 51, size=(oc, 1, 1)).astype(np.int32)
        op = relay.add(op, relay.var("bias", shape=(oc, 1, 1), dtype="int32"))
    op = _qnn_tail(op, q, op.shape, with_sum, rng, params, inputs)
    return relay.IRModule.from_expr(op), params, inputs


def dense_model(name):
    n, ic, oc, bias, with_sum, q = DENSE_PROFILES[name]
    rng = np.random.default_rng(0)
    d_zp, d_scl, k_scl = q[0], q[1], q[2]
    params, inputs = {}, {"data": rng.integers(0, 21, size=(n, ic)).astype(np.uint8)}
    params["weight"] = rng.integers(-20, 21, size=(oc, ic)).astype(np.int8)
    data = relay.var("data", shape=(n, ic), dtype="uint8")
    wgt = relay.var("weight", shape=(oc, ic), dtype="int8")
    op = relay.qnn.op.dense(data, wgt, relay.const(d_zp), relay.const(0), relay.const(np.float32(d_scl)),
                            relay.const(np.float32(k_scl)), units=oc)
    if bias:
        params["bias"] = rng.integers(-50, 51, size=(oc,)).astype(np.int32)
        op = relay.add(op, relay.var("bias", shape=(oc,), dtype="int32"))
    op = _qnn_tail(op, q, op.shape, with_sum, rng, params, inputs)
    return relay.IRModule.from_expr(op), params, inputs


def _profile(kind, name):
    return (CONV_PROFILES if kind == "conv" else DENSE_PROFILES)[name]


CASES = [("conv", k) for k in CONV_PROFILES] + [("dense", k) for k in DENSE_PROFILES]
IDS = [f"{a}-{b}" for a, b in CASES]


def _build(kind, name):
    return conv_model(name) if kind == "conv" else dense_model(name)


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_partition_constants_match_legalization(case):
    kind, name = case
    mod, params, _ = _build(kind, name)
    part = tkbyoc.partition_for_tachikoma(mod, params)
    body = part["main"].body
    assert body.op == ("tachikoma.qnn.conv2d" if kind == "conv" else "tachikoma.qnn.dense")
    prof = _profile(kind, name)
    q = prof[-1]
    with_sum = prof[-2]
    d_zp, d_scl, k_scl, rq_zp, rq_scl, sum_zp, sum_scl, o_zp, o_scl = q
    exp = tachikoma_ref.legalize_constants(
        params["weight"], params.get("bias"), d_zp, np.float32(np.float32(d_scl) * np.float32(k_scl)), 0,
        np.float32(rq_scl), rq_zp, (rq_scl, rq_zp, sum_scl, sum_zp, o_scl, o_zp) if with_sum else None)
    po = body.attrs["postops"]
    for key in ("bias", "o_scl", "act_scl", "sum_scl", "dst_zp"):
        assert np.asarray(po[key], np.float32).tobytes() == np.asarray(exp[key], np.float32).tobytes(), key
    # the composite is one op (one trace record); the chain's intermediates are gone
    plan = lower(part, params)
    assert [o.op for o in plan.ops] == [body.op]


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_composite_within_one_quantum_of_qnn(case):
    kind, name = case
    mod, params, inputs = _build(kind, name)
    ref = graph_ref.calibrate(mod, params, inputs)
    part = tkbyoc.partition_for_tachikoma(mod, params)
    got = graph_ref.calibrate(part, params, inputs)
    out_ref = ref[lower(mod, params).outputs[0]]
    out_got = got[lower(part, params).outputs[0]]
    assert out_got.dtype == out_ref.dtype == np.uint8
    diff = np.abs(out_got.astype(np.int32) - out_ref.astype(np.int32))
    assert diff.max() <= 1, f"max |composite - qnn| = {diff.max()}"


def test_unmatched_chain_is_left_alone():
    """A non-zero kernel zero point does not match the pattern (tachikoma.py:1159)."""
    rng = np.random.default_rng(3)
    w = rng.integers(-20, 21, size=(16, 8, 3, 3)).astype(np.int8)
    data = relay.var("data", shape=(1, 8, 5, 5), dtype="uint8")
    op = relay.qnn.op.conv2d(data, relay.var("weight", shape=w.shape, dtype="int8"), relay.const(0),
                             relay.const(1), relay.const(np.float32(0.2)), relay.const(np.float32(0.1)),
                             kernel_size=(3, 3), channels=16, padding=(1, 1))
    op = relay.qnn.op.requantize(op, relay.const(np.float32(0.02)), relay.const(0), relay.const(np.float32(0.2)),
                                 relay.const(30), out_dtype="int32")
    op = relay.cast(relay.clip(op, 0.0, 255.0), "uint8")
    part = tkbyoc.partition_for_tachikoma(relay.IRModule.from_expr(op), {"weight": w})
    assert part["main"].body.op == "cast"
    assert [o.op for o in lower(part, {"weight": w}).ops] == ["qnn.conv2d", "qnn.requantize", "clip", "cast"]


def test_pattern_table_names():
    assert [n for n, _ in tkbyoc.pattern_table()] == ["tachikoma.qnn.conv2d", "tachikoma.qnn.dense"]


# ------------------------------------------------------------------------------ GPU

@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_gpu_composite_bit_exact_vs_oracle(case):
    from tachikoma_amd.contrib import graph_executor
    kind, name = case
    mod, params, inputs = _build(kind, name)
    part = tkbyoc.partition_for_tachikoma(mod, params)
    for m_, tag in ((part, "composite"), (mod, "qnn")):
        exp = graph_ref.calibrate(m_, params, inputs)
        lib = relay.build(m_, target="mi355x", params=params)
        gm = graph_executor.GraphModule(lib["default"]())
        for k, v in inputs.items():
            gm.set_input(k, v)
        gm.run()
        for rec in lower(m_, params).ops:
            got = gm.get_node_output(rec.name).numpy()
            np.testing.assert_array_equal(got, exp[rec.name], err_msg=f"{tag} {rec.name} ({rec.op})")


@pytest.mark.gpu
@pytest.mark.parametrize("out_dt,sum_dt,per_channel", [("uint8", None, False), ("int8", "int8", True),
                                                        ("uint8", "uint8", True), ("int8", None, True)])
def test_gpu_postops_abi(out_dt, sum_dt, per_channel):
    """tk_tachikoma_postops through the C ABI on random int32 contractions (incl. values that
    land on .5 ties and saturate) against the oracle's post-op chain."""
    import ctypes

    import torch

    from tachikoma_amd import _lib
    rng = np.random.default_rng(11)
    n, c, h, w = 3, 24, 7, 9
    acc = rng.integers(-40000, 40000, size=(n, c, h, w)).astype(np.int32)
    acc[0, 0, 0, :4] = [1, 3, 5, 7]  # with o_scl 0.5 and bias 0 these hit exact .5 ties
    consts = {"bias": rng.uniform(-300, 300, size=c).astype(np.float32),
              "o_scl": (rng.uniform(0.001, 0.02, size=c) if per_channel else np.array([0.5])).astype(np.float32),
              "act_scl": np.float32(0.75), "sum_scl": np.float32(1.5), "dst_zp": np.float32(-3.25)}
    consts["bias"][0] = 0.0
    if per_channel:
        consts["o_scl"][0] = 0.5
    sum_src = rng.integers(0 if sum_dt == "uint8" else -128, 128, size=acc.shape).astype(sum_dt) if sum_dt else None
    exp = tachikoma_ref.postops(acc, {**consts, "o_scl": consts["o_scl"] if per_channel else consts["o_scl"][0]},
                                out_dt, sum_src=sum_src, clip=(-20.0, 200.0))
    lib = _lib.load()
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
    acc_d, bias_d, osc_d = d(acc), d(consts["bias"]), d(consts["o_scl"])
    out = torch.empty(acc.shape, dtype=torch.uint8 if out_dt == "uint8" else torch.int8, device="cuda")
    a = _lib.tk_postops_attrs()
    a.axis, a.n_scales = 1, len(consts["o_scl"])
    a.clip_lo, a.clip_hi = -20.0, 200.0
    a.act_scl, a.sum_scl, a.dst_zp = consts["act_scl"], consts["sum_scl"], consts["dst_zp"]
    a.bias, a.o_scl = bias_d.data_ptr(), osc_d.data_ptr()
    refs = [_lib.TensorRef.from_torch(t) for t in (acc_d, out)]
    sref = _lib.TensorRef.from_torch(d(sum_src)) if sum_src is not None else None
    _lib.check(lib.tk_tachikoma_postops(refs[0].ptr, sref.ptr if sref else None, refs[1].ptr, ctypes.byref(a),
                                        ctypes.c_void_p(_lib.stream_handle())), "tk_tachikoma_postops")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), exp)

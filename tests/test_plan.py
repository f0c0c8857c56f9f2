"""Host-side lowering: MRT-style naming, shapes/dtypes vs the oracle walk, fusion groups,
workload sizes."""
import numpy as np
import pytest

from oracle import graph_ref
from tachikoma_amd import relay, zoo
from tachikoma_amd.relay import qnn
from tachikoma_amd.relay.build_module import UnsupportedError, exec_groups, lower


def test_mrt_naming_post_order():
    # MRT names calls %0.. in post-order and keeps variable name_hints (mrt/symbol.py:212-253)
    x = relay.var("x", shape=(1, 4), dtype="int8")
    y = relay.var("y", shape=(1, 4), dtype="int8")
    a = relay.clip(x, -3, 3)           # %0
    b = relay.clip(y, -2, 2)           # %1
    c = qnn.op.add(a, b, 0.5, 0, 0.5, 0, 0.25, 1)  # %2
    plan = lower(relay.IRModule.from_expr(c))
    assert [o.name for o in plan.ops] == ["%0", "%1", "%2"]
    assert [o.op for o in plan.ops] == ["clip", "clip", "qnn.add"]
    assert plan.ops[2].inputs == ["%0", "%1"]
    assert [t.name for t in plan.inputs] == ["x", "y"]


def test_plan_matches_oracle_walk_lenet():
    m = zoo.lenet5(batch=2)
    plan = lower(m.mod, m.params)
    rec = graph_ref.calibrate(m.mod, m.params, {"data": m.random_input()})
    assert [t.name for t in plan.records] == list(rec)
    for t in plan.records:
        assert rec[t.name].shape == t.shape and str(rec[t.name].dtype) == t.dtype


@pytest.mark.parametrize("name,macs,ops", [("lenet5", 416520, 22), ("resnet18", 1814073344, 93),
                                           ("resnet50", 4089184256, 232), ("mobilenet_v2", 300774272, 208)])
def test_workload_sizes(name, macs, ops):
    m = zoo.MODELS[name](batch=1)
    assert zoo.macs_per_sample(m) == macs
    assert len(lower(m.mod, m.params).ops) == ops


def test_fusion_groups_resnet50():
    m = zoo.resnet50(batch=1)
    plan = lower(m.mod, m.params)
    groups = exec_groups(plan)
    blocks = [g for g in groups if g.kind == "conv_block"]
    assert len(blocks) == 53 and sum(g.kind == "dense_block" for g in groups) == 1
    covered = [o.name for g in groups for o in g.ops]
    assert sorted(covered) == sorted(o.name for o in plan.ops)      # every op exactly once
    order = {o.name: i for i, o in enumerate(plan.ops)}
    pos = {}
    for gi, g in enumerate(groups):
        for o in g.ops:
            pos[o.name] = gi
    for o in plan.ops:                                               # producers run first
        for x in o.inputs:
            if x in pos:
                assert pos[x] <= pos[o.name]
    assert len(exec_groups(plan, fuse=False)) == len(plan.ops)


def test_unsupported_paths_fail_loudly():
    m = zoo.lenet5(batch=1)
    with pytest.raises(UnsupportedError):
        relay.build(m.mod, target="llvm", params=m.params)
    # a float requantize form inside qnn.concatenate is not implemented: refused, not approximated
    a = relay.var("a", shape=(1, 4), dtype="int8")
    b = relay.var("b", shape=(1, 4), dtype="int8")
    with qnn.op.requantize_config(compute_dtype="float32"):
        y = qnn.op.concatenate(relay.Tuple([a, b]), [relay.const(0.5), relay.const(0.25)],
                               [relay.const(0), relay.const(0)], relay.const(0.5), relay.const(0), axis=1)
    with pytest.raises(UnsupportedError):
        lower(relay.IRModule.from_expr(y))
    x = relay.var("x", shape=(4,), dtype="int32")
    with pytest.raises(ValueError):
        lower(relay.IRModule.from_expr(qnn.op.requantize(x, 0.5, 0, 0.25, 0, compute_dtype="float16")))


@pytest.mark.parametrize("cd", ["float32", "float64"])
def test_float_compute_dtype_plan(cd):
    """requantize_config(compute_dtype=float32|float64) selects RequantizeLowerFP<32|64>
    (requantize.cc:392-403): the plan carries the double multipliers and the 'scaled' flag, and the
    conv blocks are not fused (their epilogue is the int64 form) -- the requantize runs alone."""
    x = relay.var("x", shape=(4,), dtype="int32")
    with qnn.op.requantize_config(compute_dtype=cd):
        y = qnn.op.requantize(x, 0.5, 0, 0.25, 0)
        y2 = qnn.op.requantize(x, 0.5, 0, 0.5, 3)
    rq = lower(relay.IRModule.from_expr(y)).ops[0]
    assert rq.attrs["compute_dtype"] == cd and rq.attrs["fp_bits"] == (32 if cd == "float32" else 64)
    assert rq.attrs["fp_scaled"] == 1 and rq.attrs["fp_multiplier"] == 2.0
    assert lower(relay.IRModule.from_expr(y2)).ops[0].attrs["fp_scaled"] == 0   # equal scales skip the multiply
    with qnn.op.requantize_config(compute_dtype=cd):
        m = zoo.lenet5(batch=1)
    plan = lower(m.mod, m.params)
    kinds = [g.kind for g in exec_groups(plan)]
    assert "conv_block" not in kinds and "dense_block" not in kinds
    assert all(o.attrs["compute_dtype"] == cd for o in plan.ops if o.op == "qnn.requantize")


def test_requantize_config_scope_resolution():
    x = relay.var("x", shape=(4,), dtype="int32")
    with qnn.op.requantize_config(rounding="TONEAREST"):
        y = qnn.op.requantize(x, 1.0, 0, 3.0, 0)
        z = qnn.op.requantize(y, 1.0, 0, 3.0, 0, rounding="UPWARD", out_dtype="int32") \
            if False else qnn.op.requantize(relay.cast(y, "int32"), 1.0, 0, 3.0, 0, rounding="UPWARD")
    plan = lower(relay.IRModule.from_expr(z))
    rq = [o for o in plan.ops if o.op == "qnn.requantize"]
    assert rq[0].attrs["rounding"] == "TONEAREST"      # config applies to "None" args
    assert rq[1].attrs["rounding"] == "UPWARD"         # explicit argument wins

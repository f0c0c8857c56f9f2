"""FuseOps grouping and fused-function naming (relay/fuse.py), host only.

Pins:
* the partitioner against the reference's own structural expectation
  (tests/python/relay/test_pass_fuse_ops.py:55-117 test_conv2d_fuse: "add can only be fused
  to z1"), written in this IR;
* stop_fusion (test_pass_fuse_ops.py:197-226) and max_depth (:580-629, relay.FuseOps.max_depth);
* ``std::hash<std::string>`` of the names te_compiler_cache.cc:234 truncates, against g++'s
  own std::hash (compiled here);
* NameSupply uniquing (name_supply.cc:75-91) and the ResNet residual join: the branch the
  post-DFS walk reaches first fuses into the add, the other keeps its own function."""
import os
import subprocess

import numpy as np
import pytest

from tachikoma_amd import relay, zoo
from tachikoma_amd.relay import fuse
from tachikoma_amd.relay.build_module import lower


def _groups(plan, **kw):
    return [[o.op if o.op != "ewise" else o.attrs["relay_op"] for o in fn.ops] for fn in fuse.fused_nodes(plan, **kw)]


def test_conv2d_fuse_reference_structure():
    dshape = (1, 16, 64, 64)
    x = relay.var("x", dshape)
    w1 = relay.var("w1", (16, 16, 3, 3))
    w2 = relay.var("w2", (16, 16, 1, 1))
    w3 = relay.var("w3", (16, 16, 3, 3))
    x1 = relay.add(x, relay.const(1.0))
    y = relay.nn.conv2d(x1, w1, padding=(1, 1))
    y1 = relay.add(y, relay.const(1.0))   # the reference writes add(const, y): same edges
    y = relay.add(y, y1)
    z2 = relay.nn.conv2d(y, w2)
    z3 = relay.nn.conv2d(y, w3, padding=(1, 1))
    z = relay.add(z2, z3)
    mod = relay.IRModule.from_expr(relay.Function(relay.free_vars(z), z))
    params = {"w1": np.zeros((16, 16, 3, 3), np.float32), "w2": np.zeros((16, 16, 1, 1), np.float32),
              "w3": np.zeros((16, 16, 3, 3), np.float32)}
    plan = lower(mod, params)
    fns = fuse.fused_nodes(plan)
    got = [[(o.op, o.inputs[1] if o.op == "nn.conv2d" else None) for o in fn.ops] for fn in fns]
    # segment 0: add; segment 1: conv(w1)+add+add; segment 2: conv(w3) alone;
    # segment 3: conv(w2) + the final add (the first branch in post order takes the add)
    assert got == [[("ewise", None)],
                   [("nn.conv2d", "w1"), ("ewise", None), ("ewise", None)],
                   [("nn.conv2d", "w3")],
                   [("nn.conv2d", "w2"), ("ewise", None)]]
    assert fns[3].inputs == [fns[1].output, "w2", fns[2].output]


def test_stop_fusion_and_max_depth():
    x = relay.var("x", (1, 8), "int32")
    y = relay.add(x, relay.const(1, "int32"))
    y = relay.stop_fusion(y)
    z = relay.add(y, relay.const(2, "int32"))
    z = relay.add(z, relay.const(3, "int32"))
    plan = lower(relay.IRModule.from_expr(relay.Function([x], z)), {})
    assert _groups(plan) == [["add"], ["annotation.stop_fusion"], ["add", "add"]]
    # relay.FuseOps.max_depth (test_fuse_max: a chain of 20 unary elementwise ops with
    # max_depth 10 is two functions of 10; 300 with the default 256 is 256 + 44)
    def chain(n):
        c = x
        for _ in range(n):
            c = relay.relu(c)
        return lower(relay.IRModule.from_expr(relay.Function([x], c)), {})
    assert [len(g) for g in _groups(chain(20), max_depth=10)] == [10, 10]
    assert [len(g) for g in _groups(chain(300))] == [256, 44]
    assert [len(g) for g in _groups(chain(5), opt_level=0)] == [1] * 5


def test_std_hash_matches_libstdcxx(tmp_path):
    names = ["", "a", "fused_qnn_conv2d", "fused_qnn_conv2d_nn_bias_add_qnn_requantize_qnn_add_clip_nn_max_pool2d_cast",
             "x" * 7, "y" * 8, "z" * 9, "fused_" + "add_" * 40]
    src = tmp_path / "h.cc"
    src.write_text('#include <functional>\n#include <iostream>\n#include <string>\nint main(){std::string s;'
                   'while(std::getline(std::cin,s)) std::cout<<std::hex<<std::hash<std::string>{}(s)<<"\\n";}\n')
    exe = tmp_path / "h"
    subprocess.run(["g++", "-O1", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], input="\n".join(names) + "\n", capture_output=True, text=True,
                         check=True).stdout.split()
    assert [f"{fuse.std_hash(n):x}" for n in names] == out


def test_candidate_name_truncation():
    short = fuse.candidate_name(["qnn.conv2d", "nn.bias_add"])
    assert short == "fused_qnn.conv2d_nn.bias_add"
    ops = ["qnn.conv2d", "nn.bias_add", "qnn.requantize", "qnn.add", "clip", "cast", "nn.max_pool2d", "qnn.requantize"]
    full = "fused" + "".join("_" + o for o in ops)
    assert len(full) > 80
    assert fuse.candidate_name(ops) == f"{full[:80]}_{fuse.std_hash(full):x}_"


def test_name_supply():
    ns = fuse.NameSupply("tvmgen_default")
    assert ns.fresh("fused_qnn.conv2d") == "tvmgen_default_fused_qnn_conv2d"
    assert ns.fresh("fused_qnn.conv2d") == "tvmgen_default_fused_qnn_conv2d_1"
    assert ns.fresh("fused_qnn.conv2d") == "tvmgen_default_fused_qnn_conv2d_2"
    nodes = fuse.NameSupply("")
    assert [nodes.fresh(n) for n in ("a", "a", "a_1")] == ["a", "a_1", "a_1_1"]


@pytest.mark.parametrize("name", ["lenet5", "resnet18", "resnet50", "mobilenet_v2"])
def test_zoo_groups(name):
    m = zoo.MODELS[name](batch=1)
    plan = lower(m.mod, m.params)
    fns = fuse.fused_nodes(plan)
    covered = [o.name for fn in fns for o in fn.ops]
    assert sorted(covered) == sorted(o.name for o in plan.ops)  # a partition of the ops
    anchors = {"qnn.conv2d", "qnn.dense", "nn.max_pool2d", "nn.avg_pool2d", "nn.global_avg_pool2d"}
    for fn in fns:
        assert sum(o.op in anchors for o in fn.ops) <= 1
        # only the group's last op is read outside the group
        inner = {o.name for o in fn.ops[:-1]}
        for other in fns:
            if other is not fn:
                assert not inner & set(x for o in other.ops for x in o.inputs)
    assert len({fn.node_name for fn in fns}) == len(fns)
    assert all(fn.func_name.startswith("tvmgen_default_fused_") for fn in fns)
    # graph order: every fused call after the calls producing its inputs
    pos = {fn.output: i for i, fn in enumerate(fns)}
    for i, fn in enumerate(fns):
        assert all(pos[x] < i for x in fn.inputs if x in pos)


def test_resnet50_residual_join():
    m = zoo.resnet50(batch=1)
    plan = lower(m.mod, m.params)
    fns = fuse.fused_nodes(plan)
    joins = [fn for fn in fns if any(o.op == "qnn.add" for o in fn.ops)]
    assert len(joins) == 16  # one per bottleneck
    for k, fn in enumerate(joins):
        # conv -> bias_add -> requantize -> qnn.add -> clip, the other operand an input; the last
        # block's output cast (before the pool anchor) joins it too
        tail = ["cast"] if k == len(joins) - 1 else []
        assert [o.op for o in fn.ops] == ["qnn.conv2d", "nn.bias_add", "qnn.requantize", "qnn.add", "clip"] + tail
        assert len(fn.inputs) == 4
    downsample = [fn for fn in fns if [o.op for o in fn.ops] == ["qnn.conv2d", "nn.bias_add", "qnn.requantize"]]
    assert len(downsample) == 4
    # distinct layers (distinct constants) get distinct functions: _1, _2, ... suffixes
    assert len({fn.func_name for fn in fns}) == len(fns)

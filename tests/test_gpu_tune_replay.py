"""Tune-table replay across library builds (DeviceModule.apply_tuning).

A find-step table names each conv block's kernel by its description, because algo numbers are plan
indices that move between builds. Blocks that have no kernel list (LeNet-5's 1 -> 6 conv: too
few channels for the MFMA path; MobileNetV2's depthwise blocks) are recorded as algo 0, the
library's own choice. Round 6 found that a table written by one build could not be replayed by
another: its algo-0 entries have no description to match ("algo 0 (not listed)"). These tests pin
the replay rules. Algo 0 replays as algo 0. Listed kernels replay by description. An unknown
description fails loudly.
"""
import copy

import numpy as np
import pytest

from tachikoma_amd import _lib, relay, zoo
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.trace_format import read_trace

pytestmark = pytest.mark.gpu


def _lenet(device):
    model = zoo.lenet5(batch=2)
    lib = relay.build(model.mod, target="mi355x", params=model.params)
    return model, lib


def test_replay_from_another_build(device, tmp_path):
    model, lib = _lenet(device)
    tuned = graph_executor.GraphModule(lib["default"](device.index, tune=True))
    table = tuned.module.tuning_table()
    algos = {tuple(e["records"]): e["algo"] for e in table["entries"]}
    assert 0 in algos.values() and any(a > 0 for a in algos.values()), table["entries"]
    other = copy.deepcopy(table)
    other["library"] = "0" * 16  # written by another build: every entry replays by its description
    replayed = graph_executor.GraphModule(lib["default"](device.index, tune=other))
    got = {tuple(e["records"]): e["algo"] for e in replayed.module.tuning}
    assert got == algos
    assert replayed.module.tune_table_digest == tuned.module.tune_table_digest
    # and the replayed module traces the same records
    x = model.random_input()
    paths = []
    for i, m in enumerate((tuned, replayed)):
        m.set_input(data=x)
        paths.append(str(tmp_path / f"t{i}.tkt"))
        m.dump_trace(paths[-1])
    a, b = (read_trace(p, copy=True).records for p in paths)
    assert set(a) == set(b)
    for name in a:
        np.testing.assert_array_equal(a[name], b[name])


def test_replay_unknown_kernel_fails(device):
    _, lib = _lenet(device)
    table = graph_executor.GraphModule(lib["default"](device.index, tune=True)).module.tuning_table()
    other = copy.deepcopy(table)
    other["library"] = "0" * 16
    listed = [e for e in other["entries"] if e["algo"] > 0]
    assert listed
    listed[0]["kernel"] = "a kernel no build of this library lists"
    with pytest.raises(_lib.TachikomaError, match="no kernel"):
        graph_executor.GraphModule(lib["default"](device.index, tune=other))

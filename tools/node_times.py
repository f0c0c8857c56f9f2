"""Per-node device time of one compute-only step (HIP events around every node,
tk_module_run_profiled), with the algorithmic bytes each node moves.  GPU only.

usage: python tools/node_times.py [model] [batch] [reps] [configs-json]

configs-json: a list of env dicts (e.g. '[{}, {"TK_ABLATE": "4"}]'); env-selected kernel
variants are read per launch, so every config is timed in this one process, interleaved.
"""
import json
import os
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, ".")
from tachikoma_amd import relay, zoo  # noqa: E402
from tachikoma_amd.contrib import graph_executor  # noqa: E402


def main(model="resnet50", batch=64, reps=5, configs=None):
    batch, reps = int(batch), int(reps)
    configs = json.loads(configs) if configs else [{}]
    m = zoo.MODELS[model](batch=batch)
    lib = relay.build(m.mod, target="mi355x", params=m.params)
    g = graph_executor.GraphModule(lib["default"](0))
    g.set_input("data", m.sample_inputs(0, batch))
    g.run()
    mod = g.module
    times = [[] for _ in configs]
    for _ in range(reps):
        for ci, cfg in enumerate(configs):
            saved = {k: os.environ.get(k) for k in cfg}
            os.environ.update(cfg)
            times[ci].append(list(mod.run_profiled().values()))
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    if len(configs) > 1:
        tc = [np.median(np.array(x), axis=0) for x in times]
        print(f"{'node':6s} {'kind':12s} " + " ".join(f"{json.dumps(c):>14s}" for c in configs))
        for i, kind in enumerate(mod.node_kinds):
            print(f"{i:<6d} {kind:12s} " + " ".join(f"{t[i] * 1e3:14.1f}" for t in tc))
        print("total  " + " " * 13 + " ".join(f"{t.sum() * 1e3:14.1f}" for t in tc))
        return
    times = times[0]
    t = np.median(np.array(times), axis=0)
    ops = {o.name: o for o in g.plan.ops}
    by_kind = defaultdict(lambda: [0, 0.0, 0])
    print(f"{'node':6s} {'kind':12s} {'desc':30s} {'us':>8s} {'GB/s':>7s}")
    for i, (recs, kind) in enumerate(zip(mod.node_records, mod.node_kinds)):
        us = t[i] * 1e3
        if recs:
            head = ops[recs[0]]
            ins = [g.plan.tensor(x) for x in head.inputs]
            nbytes = sum(x.nbytes for x in ins) + sum(ops[r].out.nbytes for r in recs)
            shp = head.out.shape
            desc = f"{head.op.split('.')[-1]} {ins[0].shape[1] if len(ins[0].shape) > 1 else ''}->" \
                   f"{shp[1] if len(shp) > 1 else ''} {'x'.join(map(str, shp[2:]))}"
        else:
            nbytes, desc = 0, "shadow"
        by_kind[kind][0] += 1
        by_kind[kind][1] += us
        by_kind[kind][2] += nbytes
        print(f"{i:<6d} {kind:12s} {desc:30s} {us:8.1f} {nbytes / max(us, 1e-3) / 1e3:7.0f}")
    print("\nby kind:")
    for k, (n, us, nb) in sorted(by_kind.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:14s} {n:4d} nodes {us:9.1f} us  {nb / max(us, 1e-3) / 1e3:7.0f} GB/s")
    print(f"total {sum(v[1] for v in by_kind.values()):.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Record sizes (bytes, one per line, trace order) of one traced step: the input of
tools/probe_copies.  usage: python tools/record_sizes.py [model=resnet50] [batch=64]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tachikoma_amd import zoo  # noqa: E402
from tachikoma_amd.relay.build_module import build  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 64
model = zoo.MODELS[name](batch=batch)
plan = build(model.mod, target="mi355x", params=model.params).plan
for t in plan.records:
    print(t.nbytes)

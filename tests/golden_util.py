"""Loader for tests/golden/qnn_kats.json (literal KATs transcribed from the reference tests)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load_array(spec):
    shape = tuple(spec["shape"])
    if "fill" in spec:
        return np.full(shape, spec["fill"], dtype=spec["dtype"])
    return np.array(spec["data"], dtype=spec["dtype"]).reshape(shape)


def load_cases(op=None):
    with open(os.path.join(HERE, "golden", "qnn_kats.json")) as f:
        doc = json.load(f)
    cases = doc["cases"]
    if op is not None:
        cases = [c for c in cases if c["op"] == op]
    return cases


def scale_const(v):
    """Python float → rank-0 float32 (per-tensor); list → 1-D float32 (per-axis)."""
    if isinstance(v, (list, tuple)):
        return np.array(v, dtype=np.float32)
    return np.float32(v)

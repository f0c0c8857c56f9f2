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


_META = r"meta\[relay\.Constant\]\[(\d+)\]"


def menangerie(name: str, seed: int = 0):
    """One of the reference's float test models (tests/golden/menangerie_<name>.relay, extracted
    from tests/python/relay/collage/menangerie.py by tools/extract_menangerie.py) parsed with seeded
    constants of the listed shapes.  The reference fills them with np.random.rand; here each one
    is drawn by its role so that activations stay bounded through 50 layers: conv / dense weights
    He-normal, batch-norm gamma and variance in [0.5, 1.5), beta, mean and biases in [-0.2, 0.2).
    Returns (IRModule, input name, input shape)."""
    import re

    from tachikoma_amd import relay
    with open(os.path.join(HERE, "golden", f"menangerie_{name}.relay")) as f:
        text = f.read()
    with open(os.path.join(HERE, "golden", f"menangerie_{name}.json")) as f:
        meta = json.load(f)
    shapes = [tuple(s) for s in meta["constant_shapes"]]
    role = {}
    for m in re.finditer(r"nn\.(conv2d|dense)\([^,]+, " + _META, text):
        role[int(m.group(2))] = "weight"
    for m in re.finditer(r"nn\.batch_norm\([^,]+, " + ", ".join([_META] * 4), text):
        for k, r in zip(range(1, 5), ("gamma", "beta", "mean", "var")):
            role[int(m.group(k))] = r
    rng = np.random.default_rng(seed)
    consts = []
    for i, shape in enumerate(shapes):
        r = role.get(i, "bias")
        if r == "weight":
            fan_in = int(np.prod(shape[1:]))
            v = rng.standard_normal(shape) * np.sqrt(2.0 / fan_in)
        elif r in ("gamma", "var"):
            v = rng.uniform(0.5, 1.5, shape)
        else:
            v = rng.uniform(-0.2, 0.2, shape)
        consts.append(v.astype(np.float32))
    mod = relay.parse(text, init_meta_table={"relay.Constant": consts})
    (iname, ishape), = meta["inputs"].items()
    return mod, iname, tuple(ishape)

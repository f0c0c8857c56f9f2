"""relay.quantize-realized graphs on the MI355X: every record of the
trace — integer shift/add/clip chains, int8 contractions, and the float32 ops the quantizer
leaves (input quantize, the skipped first conv, dequantize, pool, classifier) — bit-exact
against the oracle (oracle/realize_ref.py fixes the float summation order the kernels use)."""
import numpy as np
import pytest

from oracle import graph_ref, realize_ref
from tachikoma_amd import _lib, relay, zoo
from tachikoma_amd.contrib import graph_executor
from tachikoma_amd.relay.quantize import qconfig, quantize
from tachikoma_amd.trace_format import read_trace

from . import tk_gpu as G

pytestmark = pytest.mark.gpu


def _compare(records, expected):
    for name, exp in expected.items():
        got = records[name]
        assert got.shape == exp.shape and got.dtype == exp.dtype, (name, got.shape, exp.shape, got.dtype, exp.dtype)
        if not np.array_equal(got, exp):
            idx = tuple(np.argwhere(got != exp)[0])
            raise AssertionError(f"record {name}: first mismatch at {idx}: {got[idx]} vs {exp[idx]}")


@pytest.mark.parametrize("depth,cfg", [(18, {}), (18, {"skip_conv_layers": []}), (18, {"weight_scale": "max"}),
                                       (50, {})])
def test_realized_resnet_trace_bit_exact(device, tmp_path, depth, cfg):
    m = zoo.resnet_float(depth, batch=2, hw=64)
    with qconfig(**cfg):
        q = quantize(m.mod, m.params)
    lib = relay.build(q, target="mi355x")
    gm = graph_executor.GraphModule(lib["default"]())
    x = m.random_input()
    gm.set_input("data", x)
    path = str(tmp_path / "q.tkt")
    gm.dump_trace(path)
    tr = read_trace(path)
    exp = graph_ref.calibrate(q, {}, {"data": x})
    assert set(exp) <= set(tr.records)
    _compare(tr.records, exp)


def _ew(x, op, rhs=None, scalar=None, per_channel=False, **kw):
    out = G.empty(x.shape, str(x.dtype))
    a = _lib.tk_ewise_attrs()
    a.op = _lib.TK_EW[op]
    a.rhs_kind = (3 if per_channel else 2) if rhs is not None else (1 if scalar is not None else 0)
    if scalar is not None:
        if x.dtype == np.float32:
            a.scalar_f = float(scalar)
        else:
            a.scalar_i = int(scalar)
    a.lo, a.hi = kw.get("lo", 0.0), kw.get("hi", 0.0)
    a.multiplier, a.shift = kw.get("multiplier", 0), kw.get("shift", 0)
    dx = G.dev(x)
    dr = G.dev(rhs) if rhs is not None else None
    rc = _lib.load().tk_ewise(G.ref(dx).ptr, G.ref(dr).ptr if dr is not None else None, G.ref(out).ptr,
                              a, G.stream())
    G._sync_check(rc, f"tk_ewise {op}")
    return out.cpu().numpy()


def test_ewise_ops_bit_exact(device):
    rng = np.random.default_rng(11)
    i32 = rng.integers(-2**31, 2**31, 4099).astype(np.int32)
    i32[:4] = [2**31 - 1, -2**31, 0, -1]
    other = rng.integers(-2**31, 2**31, 4099).astype(np.int32)
    for op, s in (("add", 1 << 20), ("right_shift", 7), ("left_shift", 3), ("multiply", -3)):
        assert np.array_equal(_ew(i32, op, scalar=s), realize_ref.binary(op, i32, np.int32(s), "int32")), op
    assert np.array_equal(_ew(i32, "add", rhs=other), realize_ref.binary("add", i32, other, "int32"))
    f = (rng.standard_normal(4099) * 100).astype(np.float32)
    f[:6] = [2.5, -2.5, 0.5, -0.5, 1.5, -1.5]
    assert np.array_equal(_ew(f, "round"), realize_ref.round_away(f))
    assert np.array_equal(_ew(f, "multiply", scalar=np.float32(1 / 0.0625)), (f * np.float32(16.0)).astype(np.float32))
    assert np.array_equal(_ew(f, "clip", lo=-127.0, hi=127.0), realize_ref.clip(f, -127.0, 127.0))
    i64 = rng.integers(-2**31, 2**31, 4099).astype(np.int64)
    for m_, s_ in ((1518500250, -3), (1395864371, 1), (2**30, -2)):
        got = _ew(i64, "fixed_point_multiply", multiplier=m_, shift=s_)
        assert np.array_equal(got, realize_ref.fixed_point_multiply(i64, m_, s_)), (m_, s_)
    # int64 data beyond the int32 range: the power-of-two branch works in int64 (no wrap at 32
    # bits), the general branch multiplies the full int64 value (intrin_rule.cc:166-237)
    wide = rng.integers(-2**40, 2**40, 4099).astype(np.int64)
    for m_, s_ in ((2**30, 4), (2**30, -3), (1518500250, -3)):
        got = _ew(wide, "fixed_point_multiply", multiplier=m_, shift=s_)
        assert np.array_equal(got, realize_ref.fixed_point_multiply(wide, m_, s_)), (m_, s_)


@pytest.mark.parametrize("mode", ["kl_divergence", "percentile"])
def test_dataset_calibration_on_device(device, tmp_path, mode, monkeypatch):
    """collect_stats runs the profile graph on the MI355X; its statistics (float32 records,
    bit-exact) give the same per-layer scales as the oracle's run of the same graph, and the
    realized graph then traces bit-exact."""
    from tachikoma_amd.relay.quantize import passes
    m = zoo.resnet_float(18, batch=2, hw=64)
    data = [{"data": m.random_input(seed=s)} for s in range(2)]
    with qconfig(calibrate_mode=mode):
        q = quantize(m.mod, m.params, dataset=data)
    dev_consts = [n.data for n in relay.post_order(q["main"].body) if isinstance(n, relay.Constant)]

    def oracle_collect(mod, dataset, chunk_by=-1):
        prof, targets = passes.stats_profile(mod)
        names, c = {}, 0
        for n in relay.post_order(prof["main"].body):
            if isinstance(n, relay.Call):
                names[id(n)] = f"%{c}"
                c += 1
            elif isinstance(n, relay.Var):
                names[id(n)] = n.name_hint
        outs = [[] for _ in targets]
        for batch in dataset:
            rec = graph_ref.calibrate(prof, {}, batch)
            for j, t in enumerate(targets):
                outs[j].append(rec[names[id(t)]])
        yield [np.concatenate(o).reshape(-1) for o in outs]

    monkeypatch.setattr(passes, "collect_stats", oracle_collect)
    with qconfig(calibrate_mode=mode):
        q_ref = quantize(m.mod, m.params, dataset=data)
    ref_consts = [n.data for n in relay.post_order(q_ref["main"].body) if isinstance(n, relay.Constant)]
    assert len(dev_consts) == len(ref_consts)
    for a, b in zip(dev_consts, ref_consts):
        assert a.dtype == b.dtype and np.array_equal(a, b)
    lib = relay.build(q, target="mi355x")
    gm = graph_executor.GraphModule(lib["default"]())
    x = m.random_input(seed=7)
    gm.set_input("data", x)
    path = str(tmp_path / "q.tkt")
    gm.dump_trace(path)
    _compare(read_trace(path).records, graph_ref.calibrate(q, {}, {"data": x}))


@pytest.mark.parametrize("shape", [(64, 3, 2, 2, 1100, 3, 1, 1), (2, 6, 9, 9, 8, 3, 2, 2), (1, 4, 7, 5, 6, 1, 1, 0)])
def test_conv2d_f32_bit_exact(device, shape):
    """tk_conv2d_f32 vs the oracle's fixed-order restatement, incl. more (n, o) planes than the
    grid's y dimension holds (64 x 1100) and a grouped, strided case."""
    n, c, h, w, o, k, s, p = shape
    groups = 2 if c % 2 == 0 and o % 2 == 0 and c == 6 else 1
    rng = np.random.default_rng(12)
    x = rng.standard_normal((n, c, h, w)).astype(np.float32)
    wt = rng.standard_normal((o, c // groups, k, k)).astype(np.float32)
    oh = (h + 2 * p - k) // s + 1
    ow = (w + 2 * p - k) // s + 1
    out = G.empty((n, o, oh, ow), "float32")
    a = _lib.tk_conv2d_attrs()
    a.strides[:] = [s, s]
    a.padding[:] = [p, p, p, p]
    a.dilation[:] = [1, 1]
    a.groups = groups
    dx, dw = G.dev(x), G.dev(wt)
    G._sync_check(_lib.load().tk_conv2d_f32(G.ref(dx).ptr, G.ref(dw).ptr, G.ref(out).ptr, a, G.stream()),
                  "tk_conv2d_f32")
    exp = realize_ref.conv2d_f32(x, wt, (s, s), (p, p, p, p), (1, 1), groups)
    assert np.array_equal(out.cpu().numpy(), exp)


def test_ewise_per_channel_operand(device):
    """tk_ewise rhs_kind 3: one value per channel (axis 1) -- a batch norm's scale left unfolded
    by FoldScaleAxis -- for float32 multiply / add and the int32 wrap-around forms."""
    rng = np.random.default_rng(12)
    f = rng.standard_normal((2, 5, 7, 3)).astype(np.float32)
    s = rng.standard_normal(5).astype(np.float32)
    for op in ("multiply", "add"):
        exp = realize_ref.binary(op, f, s.reshape(5, 1, 1), "float32")
        assert np.array_equal(_ew(f, op, rhs=s, per_channel=True), exp), op
    i = rng.integers(-2**31, 2**31, (3, 4, 5, 5)).astype(np.int32)
    v = rng.integers(-2**31, 2**31, 4).astype(np.int32)
    for op in ("multiply", "add"):
        exp = realize_ref.binary(op, i, v.reshape(4, 1, 1), "int32")
        assert np.array_equal(_ew(i, op, rhs=v, per_channel=True), exp), op

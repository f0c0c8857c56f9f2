"""relay.quantize: the partition / annotate / calibrate / realize passes.

The structural checks mirror the reference's tests/python/relay/test_pass_auto_quantize.py
(test_skip_conv, test_stop_quantize, test_batch_flatten_rewrite, test_left_shift_negative,
test_dense_conv2d_rewrite).  Numerics: the realized integer graph is evaluated by the oracle
(oracle/realize_ref.py) and compared with the simulated float graph the same passes produce
with ``do_simulation=True`` (the reference's own simulation), block by block.  Parity with the
reference's realized graphs is unpinned at the bit level: no TVM build or quantize fixture is
available in this container; the passes are restated from realize.cc /
_annotate.py / _partition.py / _calibrate.py, cited per rule.
"""
import numpy as np
import pytest

from oracle import graph_ref, realize_ref
from tachikoma_amd import relay, zoo
from tachikoma_amd.relay import op as O
from tachikoma_amd.relay.build_module import UnsupportedError, exec_groups, lift_constants, lower
from tachikoma_amd.relay.fold import round_away
from tachikoma_amd.relay.quantize import qconfig, quantize


def _calls(mod):
    return [n for n in relay.post_order(mod["main"].body) if isinstance(n, relay.Call)]


def _conv_chain(depth, rng, params, x, c=8, relu_last=True):
    y = x
    for i in range(depth):
        w = relay.var(f"w{i}", (c, y.shape[1], 3, 3), "float32")
        params[f"w{i}"] = (rng.standard_normal((c, y.shape[1], 3, 3)) * np.sqrt(2 / (9 * y.shape[1]))).astype(np.float32)
        y = O.conv2d(y, w, padding=1)
        if relu_last or i < depth - 1:
            y = O.relu(y)
    return y


def test_skip_conv():
    rng = np.random.default_rng(0)
    params = {}
    x = relay.var("data", (1, 16, 16, 16), "float32")
    y = _conv_chain(2, rng, params, x, c=16)
    mod = relay.IRModule.from_expr(y)
    for skip in ([], [0], [1], [0, 1], None):
        with qconfig(skip_conv_layers=skip):
            q = quantize(mod, params)
        convs = [n for n in _calls(q) if n.op == "nn.conv2d"]
        assert len(convs) == 2
        for i, cv in enumerate(convs):
            skipped = skip is not None and i in skip
            want = ("float32", "float32", "float32") if skipped else ("int8", "int8", "int32")
            assert (cv.args[0].dtype, cv.args[1].dtype, cv.dtype) == want, (skip, i)


def test_stop_quantize():
    rng = np.random.default_rng(1)
    params = {}
    x = relay.var("data", (1, 16, 16, 16), "float32")
    y = _conv_chain(1, rng, params, x, c=16)
    p = O.global_avg_pool2d(y)
    w = relay.var("w1", (16, 16, 1, 1), "float32")
    params["w1"] = rng.standard_normal((16, 16, 1, 1)).astype(np.float32)
    out = O.relu(O.conv2d(p, w))
    with qconfig(skip_conv_layers=[]):
        q = quantize(relay.IRModule.from_expr(out), params)
    convs = [n for n in _calls(q) if n.op == "nn.conv2d"]
    assert convs[0].dtype == "int32" and convs[1].dtype == "float32"  # nothing quantized after the pool
    gap = [n for n in _calls(q) if n.op == "nn.global_avg_pool2d"][0]
    assert gap.args[0].dtype == "int32"  # AvgPoolRealize casts to the activation dtype


def test_batch_flatten_rewrite():
    rng = np.random.default_rng(2)
    params = {}
    x = relay.var("data", (1, 16, 8, 8), "float32")
    y = O.batch_flatten(_conv_chain(1, rng, params, x, c=16, relu_last=False))
    with qconfig(skip_conv_layers=[]):
        q = quantize(relay.IRModule.from_expr(y), params)
    bf = [n for n in _calls(q) if n.op == "nn.batch_flatten"]
    assert bf and all(n.dtype == "int8" for n in bf)


def test_left_shift_negative():
    x = relay.var("data", (1, 16, 8, 8), "float32")
    w = relay.const(np.full((16, 16, 3, 3), 256.0, np.float32))
    q = None
    with qconfig(calibrate_mode="global_scale", global_scale=8.0, skip_conv_layers=None):
        q = quantize(relay.IRModule.from_expr(O.relu(O.conv2d(x, w, padding=1))))
    shifts = [n for n in _calls(q) if n.op == "left_shift"]
    assert shifts, 'Broken case, can\'t find any "left_shift" operators.'
    for s in shifts:
        assert int(s.args[1].data) >= 0


def test_dense_conv2d_rewrite():
    rng = np.random.default_rng(3)
    inp = relay.var("inp", (1, 64), "float32")
    dense = O.bias_add(O.dense(inp, relay.const(rng.random((4, 64)).astype(np.float32))),
                       relay.const(rng.random(4).astype(np.float32)))
    data = relay.var("data", (1, 16, 8, 8), "float32")
    conv = O.conv2d(data, relay.const(rng.random((16, 16, 3, 3)).astype(np.float32)), padding=1)
    with qconfig(calibrate_mode="global_scale", global_scale=8.0, skip_dense_layer=False):
        qd = quantize(relay.IRModule.from_expr(dense))
        qc = quantize(relay.IRModule.from_expr(conv))
    d = [n for n in _calls(qd) if n.op == "nn.dense"][0]
    assert (d.args[0].dtype, d.args[1].dtype, d.dtype) == ("int8", "int8", "int32")
    c = [n for n in _calls(qc) if n.op == "nn.conv2d"][0]  # conv 0 is skipped by default
    assert (c.args[0].dtype, c.args[1].dtype, c.dtype) == ("float32", "float32", "float32")


@pytest.mark.parametrize("weight_scale", ["power2", "max"])
def test_realized_matches_simulation_per_block(weight_scale):
    """Realized integer graph vs the simulated float graph (do_simulation=True): equal for conv
    chains; a residual join may differ by one activation quantum (2^-4 at global_scale 8), where
    the simulation's round-half-away meets the realized shift's round-half-up."""
    rng = np.random.default_rng(4)
    params = {}
    x = relay.var("data", (2, 4, 8, 8), "float32")
    y = _conv_chain(2, rng, params, x)
    w = relay.var("wr", (8, 8, 3, 3), "float32")
    params["wr"] = (rng.standard_normal((8, 8, 3, 3)) * 0.15).astype(np.float32)
    res = O.relu(O.add(O.conv2d(y, w, padding=1), y))
    data = rng.standard_normal((2, 4, 8, 8)).astype(np.float32)
    for expr, tol in ((y, 0.0), (res, 2.0 ** -4)):
        mod = relay.IRModule.from_expr(expr)
        with qconfig(skip_conv_layers=[], do_simulation=True, weight_scale=weight_scale):
            s = quantize(mod, params)
        with qconfig(skip_conv_layers=[], weight_scale=weight_scale):
            q = quantize(mod, params)
        so = list(graph_ref.calibrate(s, {}, {"data": data}).values())[-1]
        qo = list(graph_ref.calibrate(q, {}, {"data": data}).values())[-1]
        assert qo.dtype == np.float32 and qo.shape == so.shape
        assert np.abs(so - qo).max() <= tol + 1e-7


def test_weight_scale_max_uses_fixed_point_multiply():
    rng = np.random.default_rng(5)
    params = {}
    x = relay.var("data", (1, 4, 8, 8), "float32")
    y = _conv_chain(2, rng, params, x)
    with qconfig(skip_conv_layers=[], weight_scale="max"):
        q = quantize(relay.IRModule.from_expr(y), params)
    ops = [n.op for n in _calls(q)]
    assert "fixed_point_multiply" in ops
    fpm = [n for n in _calls(q) if n.op == "fixed_point_multiply"]
    assert all(n.args[0].dtype in ("int32", "int64") for n in fpm)


def test_resnet_realized_graph_lowers_to_device_ops():
    m = zoo.resnet_float(18, batch=1, hw=64)
    for cfg in ({}, {"skip_conv_layers": []}):
        with qconfig(**cfg):
            q = quantize(m.mod, m.params)
        mod, params = lift_constants(q, {})
        plan = lower(mod, params)
        ops = {o.op for o in plan.ops}
        assert "qnn.conv2d" in ops and "ewise" in ops and "nn.dense" in ops  # float classifier (skip_dense_layer)
        assert ("nn.conv2d" in ops) == (cfg == {})  # float first conv only when skipped
        assert all(p.name.startswith("_const") for p in plan.params)
        assert len(exec_groups(plan)) == len(plan.ops)  # no QNN block pattern in a realized graph
        int_convs = [o for o in plan.ops if o.op == "qnn.conv2d"]
        assert all(o.attrs["relay_op"] == "nn.conv2d" and o.attrs["input_zero_point"] == 0 for o in int_convs)


def test_unsupported_modes_fail_loudly():
    x = relay.var("data", (1, 4, 8, 8), "float32")
    params = {}
    y = _conv_chain(1, np.random.default_rng(6), params, x)
    with pytest.raises(ValueError):
        with qconfig(calibrate_mode="kl_divergence"):
            quantize(relay.IRModule.from_expr(y), params)  # needs a dataset
    with pytest.raises(ValueError):
        with qconfig(partition_conversions="sometimes"):
            quantize(relay.IRModule.from_expr(y), params)
    with pytest.raises(AttributeError):
        qconfig(no_such_field=1)


# ---- partition_conversions (python/tvm/relay/quantize/_partition_conversions.py), the structure
# and the partitioned-vs-unpartitioned agreement of test_pass_auto_quantize.py:178-330

BASE_CFG = {"skip_conv_layers": [], "skip_dense_layer": False, "dtype_input": "int8", "dtype_weight": "int8",
            "dtype_activation": "int32"}


def _eval(expr, params, inputs):
    """The value of ``expr`` over graph inputs / params (oracle walker); tuples field by field."""
    from tachikoma_amd.relay.expr import Tuple
    if isinstance(expr, Tuple):
        return [_eval(f, params, inputs) for f in expr.fields]
    if isinstance(expr, relay.Var):
        return inputs[expr.name_hint] if expr.name_hint in inputs else params[expr.name_hint]
    mod = relay.IRModule.from_expr(expr)
    names = {v.name_hint for v in mod["main"].params}
    recs = graph_ref.calibrate(mod, {k: v for k, v in params.items() if k in names},
                               {k: v for k, v in inputs.items() if k in names})
    return list(recs.values())[-1]


def _verify_partition(mod, params, inputs):
    from tachikoma_amd.relay.expr import Tuple
    with qconfig(**BASE_CFG, partition_conversions="disabled"):
        un = quantize(mod, params)
    assert un.get_global_vars() == ["main"]
    with qconfig(**BASE_CFG, partition_conversions="fully_integral"):
        part = quantize(mod, params)
    assert set(part.get_global_vars()) == {"main", "quantize_inputs", "quantized_main", "dequantize_outputs"}
    pre, mid, post = part["quantize_inputs"], part["quantized_main"], part["dequantize_outputs"]
    assert isinstance(pre.body, Tuple) and len(pre.body.fields) == len(mid.params)
    ops = lambda f: {n.op for n in relay.post_order(f.body) if isinstance(n, relay.Call)}  # noqa: E731
    assert ops(pre) <= {"add", "multiply", "right_shift", "clip", "round", "cast"}
    assert ops(post) <= {"add", "multiply", "right_shift", "clip", "round", "cast"}
    assert {n.dtype for n in relay.post_order(mid.body) if isinstance(n, (relay.Call, relay.Var))} <= \
        {"int8", "int32"}
    want = _eval(un["main"].body, params, inputs)
    # main (the composition) and the three partitions run one after another agree with the
    # unpartitioned result
    np.testing.assert_array_equal(_eval(part["main"].body, params, inputs), want)
    staged = dict(zip([p.name_hint for p in mid.params], _eval(pre.body, params, inputs)))
    core = _eval(mid.body, params, staged)
    np.testing.assert_array_equal(_eval(post.body, params, {post.params[0].name_hint: core}), want)
    return part


def test_partition_conversions_conv2d():
    rng = np.random.default_rng(21)
    x = relay.var("x", (1, 4, 16, 16), "float32")
    w = relay.var("w", (4, 4, 3, 3), "float32")
    y = relay.nn.conv2d(x, w, padding=(1, 1, 1, 1), channels=4, kernel_size=(3, 3))
    params = {"w": rng.uniform(0, 1, (4, 4, 3, 3)).astype(np.float32)}
    part = _verify_partition(relay.IRModule.from_expr(y), params,
                             {"x": rng.uniform(0, 1, (1, 4, 16, 16)).astype(np.float32)})
    # the partitioned main builds like any quantized graph
    from tachikoma_amd.relay.build_module import build
    assert build(part, params={}).plan.ops


def test_partition_conversions_multiple_args():
    rng = np.random.default_rng(22)
    xs = [relay.var(f"x{i}", (1, 4, 16, 16), "float32") for i in (1, 2)]
    ws = [relay.var(f"w{i}", (4, 4, 3, 3), "float32") for i in (1, 2)]
    convs = [relay.nn.conv2d(x, w, padding=(1, 1, 1, 1), channels=4, kernel_size=(3, 3)) for x, w in zip(xs, ws)]
    y = relay.add(*convs)
    params = {f"w{i}": rng.uniform(0, 1, (4, 4, 3, 3)).astype(np.float32) for i in (1, 2)}
    part = _verify_partition(relay.IRModule.from_expr(y), params,
                             {f"x{i}": rng.uniform(0, 1, (1, 4, 16, 16)).astype(np.float32) for i in (1, 2)})
    assert len(part["quantized_main"].params) == 2


def test_partition_conversions_fails_when_not_integral():
    """verify_partition_fails (test_pass_auto_quantize.py:198-209): 'enabled' always partitions;
    'fully_integral' asserts when a partition is not a pure conversion / integer one."""
    x = relay.var("x", (10, 10), "float32")
    y = relay.var("y", (10, 10), "float32")
    mod = relay.IRModule.from_expr(relay.add(x, y))
    with qconfig(**BASE_CFG, partition_conversions="enabled"):
        part = quantize(mod, {})
    assert "quantized_main" in part.get_global_vars()
    with pytest.raises(AssertionError):
        with qconfig(**BASE_CFG, partition_conversions="fully_integral"):
            quantize(mod, {})


def test_round_away_and_oracle_agree_on_ties():
    v = np.array([-2.5, -1.5, -0.5, 0.5, 1.5, 2.5, 0.49999997, -0.49999997, 1e8 + 0.5, -3.0], np.float32)
    want = np.array([-3, -2, -1, 1, 2, 3, 0, 0, 1e8, -3], np.float32)
    assert np.array_equal(round_away(v), want)
    assert np.array_equal(realize_ref.round_away(v), want)


def test_fold_constant_matches_oracle_ops():
    from tachikoma_amd.relay.fold import eval_const_call
    rng = np.random.default_rng(7)
    a = rng.integers(-2**31, 2**31, 64).astype(np.int32)
    for op, b in (("add", np.int32(123456789)), ("left_shift", np.int32(3)), ("right_shift", np.int32(5)),
                  ("multiply", np.int32(-7))):
        call = getattr(O, op)(relay.const(a), relay.const(b))
        assert np.array_equal(eval_const_call(call, [a, b]), realize_ref.binary(op, a, b, "int32"))


def test_realized_graph_text_round_trip():
    """IRModule.astext -> relay.parse of a realized graph: same
    ops, same oracle records."""
    m = zoo.resnet_float(18, batch=1, hw=32)
    with qconfig(weight_scale="max"):
        q = quantize(m.mod, m.params)
    q2 = relay.parse(q.astext())
    assert [n.op for n in _calls(q2)] == [n.op for n in _calls(q)]
    x = m.random_input()
    r1 = graph_ref.calibrate(q, {}, {"data": x})
    r2 = graph_ref.calibrate(q2, {}, {"data": x})
    assert list(r1) == list(r2)
    for k in r1:
        assert np.array_equal(r1[k], r2[k]), k
    f2 = relay.parse(m.mod.astext())  # the float input graph too
    assert [n.op for n in _calls(f2)] == [n.op for n in _calls(m.mod)]


def test_kl_threshold_matches_restatement():
    """tk_find_scale_by_kl (native MinimizeKL) vs the oracle's scalar float32 restatement."""
    import ctypes
    from tachikoma_amd import _lib
    from tachikoma_amd.relay.quantize.passes import find_scale_by_kl
    rng = np.random.default_rng(8)
    for dist in (rng.standard_normal(5000), np.abs(rng.standard_normal(5000)), rng.laplace(size=5000) * 3):
        arr = dist.astype(np.float32)
        thres = max(abs(arr.min()), abs(arr.max()))
        hist, edges = np.histogram(arr, bins=101, range=(-thres, thres))
        assert edges.dtype == np.float32  # numpy keeps the data's float32 (the C side reads float*)
        h = np.ascontiguousarray(hist, np.int32)
        out = ctypes.c_float()
        _lib.check(_lib.load().tk_find_scale_by_kl(h.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                   edges.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 101, 11,
                                                   ctypes.byref(out)), "kl")
        assert np.float32(out.value) == np.float32(realize_ref.minimize_kl(hist, edges, 101, 11))
        t = find_scale_by_kl(arr)  # full size: 8001 bins, 255 buckets
        assert 0 < t <= thres * 1.0001


def test_percentile_scale():
    from tachikoma_amd.relay.quantize.passes import find_scale_by_percentile
    arr = np.arange(-100000, 100000, dtype=np.float32)
    assert find_scale_by_percentile(arr) == np.sort(np.abs(arr))[int(arr.size * 0.99999)]


@pytest.mark.parametrize("mode", ["kl_divergence", "percentile"])
def test_dataset_calibration_order(monkeypatch, mode):
    """Dataset modes consume one scale per non-weight simulated_quantize, in post-order (the
    order collect_stats profiles them); the stats here come from the oracle run of the profile
    graph (the device run is tests/test_gpu_realize.py)."""
    from tachikoma_amd.relay.quantize import passes
    m = zoo.resnet_float(18, batch=1, hw=32)
    data = [{"data": m.random_input(seed=s)} for s in range(2)]

    def fake_collect(mod, dataset, chunk_by=-1):
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

    monkeypatch.setattr(passes, "collect_stats", fake_collect)
    with qconfig(calibrate_mode=mode, skip_conv_layers=[]):
        q = quantize(m.mod, m.params, dataset=data)
    with qconfig(calibrate_mode=mode, skip_conv_layers=[], do_simulation=True):
        s = quantize(m.mod, m.params, dataset=data)
    sq = [n for n in _calls(s) if n.op == passes.SQ]
    kinds = [n.attrs["kind"] for n in sq]
    scales = [float(n.args[1].data) for n in sq]
    assert len(set(scales)) > 3  # per-layer scales, not one global scale
    assert any(k != 2 for k in kinds)
    out = list(graph_ref.calibrate(q, {}, {"data": data[0]["data"]}).values())[-1]
    assert out.dtype == np.float32 and np.isfinite(out).all()


def test_fixed_point_multiply_int64_power_of_two_kat():
    """relay.fixed_point_multiply on int64 data: the power-of-two branch of the
    q_multiply_shift legalization (intrin_rule.cc:223-237) shifts and rounds in x's dtype, so
    int64 values beyond the int32 range do not wrap; the general branch (:166-195) casts the
    int64 product's result to int32."""
    from oracle import realize_ref
    x = np.array([2**35 + 3, -(2**35) - 9, 5, -5], np.int64)
    assert realize_ref.fixed_point_multiply(x, 1 << 30, 4).tolist() == [2**38 + 24, -(2**38) - 72, 40, -40]
    assert realize_ref.fixed_point_multiply(x, 1 << 30, -3).tolist() == [2**31, -(2**31) - 1, 0, 0]
    # general branch: (x * m + 2^(30+rs)) >> (31+rs) in int64 (wrapping at 64 bits), then int32
    m, s = 1518500250, -3

    def wrap(v, bits):
        return ((v + 2**(bits - 1)) % 2**bits) - 2**(bits - 1)
    exp = [wrap(wrap(wrap(int(v) * m, 64) + (1 << 33), 64) >> 34, 32) for v in x]
    assert realize_ref.fixed_point_multiply(x, m, s).tolist() == exp


def test_kl_histogram_edges_are_float32():
    """kl_divergence.py:46-48 hands np.histogram's edges to MinimizeKL as c_float*: for the
    float32 statistics the profile graph produces, numpy builds float32 edges (result_type of
    the float32 range and data), so the reference's cast reads real float32 edges and
    find_scale_by_kl's explicit float32 conversion is the identity."""
    arr = np.random.default_rng(0).standard_normal(10000).astype(np.float32)
    thres = max(abs(np.min(arr)), abs(np.max(arr)))
    _, edges = np.histogram(arr, bins=8001, range=(-thres, thres))
    assert edges.dtype == np.float32


def test_kl_edges_reference_byte_buffer():
    """find_scale_by_kl hands MinimizeKL the bytes the reference's c_float* cast of np.histogram's
    edges would (kl_divergence.py:46-51): identical to the values for float32 statistics, the
    first num_bins + 1 float32 words of the float64 buffer for float64 statistics; edges_as="values"
    converts the float64 edges instead."""
    import ctypes
    from tachikoma_amd import _lib
    from tachikoma_amd.relay.quantize.passes import find_scale_by_kl, kl_edge_buffer
    rng = np.random.default_rng(9)
    nb, nq = 201, 21
    for dt in (np.float32, np.float64):
        arr = (rng.standard_normal(20000) * 2.5).astype(dt)
        thres = max(abs(np.min(arr)), abs(np.max(arr)))
        hist, edges = np.histogram(arr, bins=nb, range=(-thres, thres))
        assert edges.dtype == dt
        buf = kl_edge_buffer(edges, nb)
        # the reference's buffer, built the way its ctypes cast builds it
        cbuf = ctypes.cast(edges.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.POINTER(ctypes.c_float))
        assert np.array_equal(buf.view(np.uint32), np.array([cbuf[i] for i in range(nb + 1)], np.float32).view(np.uint32))
        if dt == np.float32:
            assert np.array_equal(buf, edges)
        exp = np.float32(realize_ref.minimize_kl(hist, buf, nb, nq))
        assert np.float32(find_scale_by_kl(arr, num_bins=nb, num_quantized_bins=nq)) == exp
        got_v = np.float32(find_scale_by_kl(arr, num_bins=nb, num_quantized_bins=nq, edges_as="values"))
        assert got_v == np.float32(realize_ref.minimize_kl(hist, edges.astype(np.float32), nb, nq))
        if dt == np.float32:
            assert got_v == exp
    with pytest.raises(ValueError):
        find_scale_by_kl(np.ones(10, np.float32), edges_as="bogus")

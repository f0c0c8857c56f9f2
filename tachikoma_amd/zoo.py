"""Deterministic synthetic int8 QNN workloads (BASELINE.json configs).

No pretrained weights or datasets are reachable (no network), so each model is
built from its standard topology with seeded synthetic parameters:

* activations at the input: int8 uniform on [-128, 127];
* weights: int8 uniform on [-128, 127], kernel zero point 0, per-output-channel
  scale ``s_w[c] = (32/σ_acc) · U[0.2, 1.8]`` (a 9x spread across channels, normalised
  so output scales stay O(input scale) through 50+ layers instead of overflowing float32);
* per-layer input zero point uniform on [-8, 8];
* bias: int32 uniform on [-2^14, 2^14];
* requantize: per-channel ``input_scale = s_a · s_w[c]`` (float32), ``output_scale``
  chosen analytically so the int8 output has a standard deviation of about 32
  for the mean channel (s_out = s_a · mean(s_w) · σ_acc / 32 with
  σ_acc = sqrt(K) · σ_a · 73.9): per-channel multipliers M[c] = s_w[c]/mean(s_w) · 32/σ_acc
  give int8 outputs with std 6..58, spread over the int8 range without saturating
  every channel.

Each conv/dense layer is ``qnn.conv2d|qnn.dense → nn.bias_add → qnn.requantize(axis=1)
→ clip`` (clip = ReLU/ReLU6 in the quantised domain), the Relay QNN form the
reference's TFLite/PyTorch importers produce.  Residual joins use ``qnn.add``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import relay
from .relay import qnn

SIGMA_W = 73.9  # std of uniform int8 on [-128, 127]


@dataclass
class Model:
    name: str
    mod: relay.IRModule
    params: Dict[str, np.ndarray]
    input_name: str
    input_shape: Tuple[int, ...]
    input_dtype: str
    seed: int

    def random_input(self, seed: Optional[int] = None, batch: Optional[int] = None) -> np.ndarray:
        rng = np.random.default_rng(self.seed + 1000 if seed is None else seed)
        shape = list(self.input_shape)
        if batch is not None:
            shape[0] = batch
        return rng.integers(-128, 128, size=shape, dtype=np.int64).astype(self.input_dtype)

    def sample_inputs(self, offset: int, count: int, seed: Optional[int] = None) -> np.ndarray:
        """Samples [offset, offset+count) of the global synthetic batch; sample i depends only
        on (seed, i), so a shard's content does not depend on how the batch is split."""
        base = self.seed + 1000 if seed is None else seed
        shape = list(self.input_shape)
        shape[0] = 1
        out = [np.random.default_rng([base, offset + i]).integers(-128, 128, size=shape, dtype=np.int64)
               for i in range(count)]
        return np.concatenate(out, axis=0).astype(self.input_dtype) if out else \
            np.zeros([0] + shape[1:], self.input_dtype)


class _Builder:
    def __init__(self, seed: int):
        self.rng = np.random.default_rng(seed)
        self.params: Dict[str, np.ndarray] = {}

    def weight(self, name: str, shape) -> relay.Var:
        w = self.rng.integers(-128, 128, size=shape, dtype=np.int64).astype(np.int8)
        self.params[name] = w
        return relay.var(name, shape=shape, dtype="int8")

    def bias(self, name: str, n: int) -> relay.Var:
        b = self.rng.integers(-(1 << 14), (1 << 14) + 1, size=(n,), dtype=np.int64).astype(np.int32)
        self.params[name] = b
        return relay.var(name, shape=(n,), dtype="int32")

    def zp(self) -> int:
        return int(self.rng.integers(-8, 9))

    def wscale(self, n: int, k: int, sigma_a: float) -> np.ndarray:
        base = 32.0 / (math.sqrt(max(k, 1)) * max(sigma_a, 1.0) * SIGMA_W)
        return (base * self.rng.uniform(0.2, 1.8, size=n)).astype(np.float32)


@dataclass
class QTensor:
    """An int8 activation with its quantisation parameters (what the next layer needs)."""
    expr: relay.Expr
    scale: float
    zp: int
    sigma: float  # estimated int8 std (for the analytic output scale)


def _requant_out_scale(s_a: float, s_w: np.ndarray, k: int, sigma_a: float, target: float = 32.0) -> float:
    sigma_acc = math.sqrt(max(k, 1)) * max(sigma_a, 1.0) * SIGMA_W
    return float(np.float32(s_a * float(np.mean(s_w)) * sigma_acc / target))


def conv_block(b: _Builder, x: QTensor, name: str, cout: int, k: int, stride: int = 1, pad: int = 0,
               groups: int = 1, act: Optional[str] = "relu") -> QTensor:
    cin = x.expr.shape[1]
    w = b.weight(f"{name}.weight", (cout, cin // groups, k, k))
    bias = b.bias(f"{name}.bias", cout)
    s_w = b.wscale(cout, (cin // groups) * k * k, x.sigma)
    conv = qnn.op.conv2d(x.expr, w, relay.const(x.zp, "int32"), relay.const(0, "int32"),
                         relay.const(x.scale, "float32"), relay.const(s_w, "float32"), kernel_size=(k, k),
                         channels=cout, strides=(stride, stride), padding=(pad, pad), groups=groups)
    y = relay.nn.bias_add(conv, bias, axis=1)
    s_in = (np.float32(x.scale) * s_w).astype(np.float32)
    s_out = _requant_out_scale(x.scale, s_w, (cin // groups) * k * k, x.sigma)
    zp_out = b.zp()
    y = qnn.op.requantize(y, relay.const(s_in, "float32"), relay.const(0, "int32"),
                          relay.const(s_out, "float32"), relay.const(zp_out, "int32"), axis=1, out_dtype="int8")
    sigma = 32.0
    if act == "relu":
        y = relay.clip(y, float(zp_out), 127.0)
        sigma = 20.0
    elif act == "relu6":
        y = relay.clip(y, float(zp_out), float(min(127, zp_out + 96)))
        sigma = 20.0
    return QTensor(y, s_out, zp_out, sigma)


def dense_block(b: _Builder, x: QTensor, name: str, units: int, act: Optional[str] = "relu") -> QTensor:
    k = x.expr.shape[1]
    w = b.weight(f"{name}.weight", (units, k))
    bias = b.bias(f"{name}.bias", units)
    s_w = b.wscale(units, k, x.sigma)
    d = qnn.op.dense(x.expr, w, relay.const(x.zp, "int32"), relay.const(0, "int32"),
                     relay.const(x.scale, "float32"), relay.const(s_w, "float32"), units=units)
    y = relay.nn.bias_add(d, bias, axis=1)
    s_in = (np.float32(x.scale) * s_w).astype(np.float32)
    s_out = _requant_out_scale(x.scale, s_w, k, x.sigma)
    zp_out = b.zp()
    y = qnn.op.requantize(y, relay.const(s_in, "float32"), relay.const(0, "int32"),
                          relay.const(s_out, "float32"), relay.const(zp_out, "int32"), axis=1, out_dtype="int8")
    sigma = 32.0
    if act == "relu":
        y = relay.clip(y, float(zp_out), 127.0)
        sigma = 20.0
    return QTensor(y, s_out, zp_out, sigma)


def qadd(b: _Builder, x: QTensor, y: QTensor, relu: bool = True) -> QTensor:
    s_c = float(np.float32(max(x.scale, y.scale) * 1.5))
    zp_c = b.zp()
    z = qnn.op.add(x.expr, y.expr, relay.const(x.scale, "float32"), relay.const(x.zp, "int32"),
                   relay.const(y.scale, "float32"), relay.const(y.zp, "int32"), relay.const(s_c, "float32"),
                   relay.const(zp_c, "int32"))
    if relu:
        z = relay.clip(z, float(zp_c), 127.0)
    return QTensor(z, s_c, zp_c, 24.0)


def _input(b: _Builder, shape) -> QTensor:
    x = relay.var("data", shape=shape, dtype="int8")
    return QTensor(x, 0.0235, b.zp(), 73.9)


def _finish(name, b, out: QTensor, shape, seed) -> Model:
    mod = relay.IRModule.from_expr(out.expr)
    return Model(name, mod, b.params, "data", tuple(shape), "int8", seed)


def _head(b: _Builder, x: QTensor, classes: int = 1000) -> QTensor:
    y = relay.cast(x.expr, "int32")
    y = relay.nn.global_avg_pool2d(y)
    y = relay.cast(y, "int8")
    y = relay.nn.batch_flatten(y)
    return dense_block(b, QTensor(y, x.scale, x.zp, x.sigma), "fc", classes, act=None)


# ---------------------------------------------------------------- configs

def qnn_dense_128(seed: int = 0) -> Model:
    """Config 1: qnn.dense [128,128] x [128,128]^T, zp_a=-3, s_a=0.05, s_w=0.01, bias, requantize
    (s_in = s_a*s_w, zp_in 0, s_out 0.1, zp_out 5, int8)."""
    rng = np.random.default_rng(seed)
    data_np = rng.integers(-128, 128, size=(128, 128), dtype=np.int64).astype(np.int8)  # input drawn first
    w = rng.integers(-128, 128, size=(128, 128), dtype=np.int64).astype(np.int8)
    bias = rng.integers(-1000, 1001, size=(128,), dtype=np.int64).astype(np.int32)
    x = relay.var("data", shape=(128, 128), dtype="int8")
    wv = relay.var("weight", shape=(128, 128), dtype="int8")
    bv = relay.var("bias", shape=(128,), dtype="int32")
    d = qnn.op.dense(x, wv, relay.const(-3, "int32"), relay.const(0, "int32"), relay.const(0.05, "float32"),
                     relay.const(0.01, "float32"), units=128)
    y = relay.nn.bias_add(d, bv)
    y = qnn.op.requantize(y, relay.const(np.float32(np.float32(0.05) * np.float32(0.01)), "float32"),
                          relay.const(0, "int32"), relay.const(0.1, "float32"), relay.const(5, "int32"),
                          out_dtype="int8")
    m = Model("qnn_dense_128", relay.IRModule.from_expr(y), {"weight": w, "bias": bias}, "data", (128, 128), "int8",
              seed)
    m.fixed_input = data_np
    return m


def lenet5(batch: int = 1, seed: int = 1) -> Model:
    """Config 2: LeNet-5 int8, [B,1,28,28] (416,520 MAC/sample)."""
    b = _Builder(seed)
    x = _input(b, (batch, 1, 28, 28))
    x = conv_block(b, x, "conv1", 6, 5, pad=2)
    x = QTensor(relay.nn.max_pool2d(x.expr, pool_size=(2, 2), strides=(2, 2)), x.scale, x.zp, x.sigma)
    x = conv_block(b, x, "conv2", 16, 5)
    x = QTensor(relay.nn.max_pool2d(x.expr, pool_size=(2, 2), strides=(2, 2)), x.scale, x.zp, x.sigma)
    x = QTensor(relay.nn.batch_flatten(x.expr), x.scale, x.zp, x.sigma)
    x = dense_block(b, x, "fc1", 120)
    x = dense_block(b, x, "fc2", 84)
    x = dense_block(b, x, "fc3", 10, act=None)
    return _finish("lenet5", b, x, (batch, 1, 28, 28), seed)


def _resnet_stem(b: _Builder, batch: int, hw: int) -> QTensor:
    x = _input(b, (batch, 3, hw, hw))
    x = conv_block(b, x, "conv1", 64, 7, stride=2, pad=3)
    return QTensor(relay.nn.max_pool2d(x.expr, pool_size=(3, 3), strides=(2, 2), padding=(1, 1)), x.scale, x.zp,
                   x.sigma)


def resnet18(batch: int = 64, seed: int = 2, hw: int = 224) -> Model:
    """Config 3: torchvision ResNet-18 topology (BasicBlock [2,2,2,2]), BN folded."""
    b = _Builder(seed)
    x = _resnet_stem(b, batch, hw)
    cin = 64
    for li, (cout, blocks, stride) in enumerate(((64, 2, 1), (128, 2, 2), (256, 2, 2), (512, 2, 2))):
        for bi in range(blocks):
            s = stride if bi == 0 else 1
            pre = f"layer{li + 1}.{bi}"
            y = conv_block(b, x, f"{pre}.conv1", cout, 3, stride=s, pad=1)
            y = conv_block(b, y, f"{pre}.conv2", cout, 3, stride=1, pad=1, act=None)
            sc = x
            if s != 1 or cin != cout:
                sc = conv_block(b, x, f"{pre}.downsample", cout, 1, stride=s, act=None)
            x = qadd(b, y, sc)
            cin = cout
    return _finish("resnet18", b, _head(b, x), (batch, 3, hw, hw), seed)


def resnet50(batch: int = 64, seed: int = 3, hw: int = 224) -> Model:
    """Config 4: ResNet-50 bottleneck [3,4,6,3] (torchvision layout: stride on the 3x3 conv),
    4,089,184,256 MAC/sample at 224x224."""
    b = _Builder(seed)
    x = _resnet_stem(b, batch, hw)
    cin = 64
    for li, (width, blocks, stride) in enumerate(((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))):
        cout = width * 4
        for bi in range(blocks):
            s = stride if bi == 0 else 1
            pre = f"layer{li + 1}.{bi}"
            y = conv_block(b, x, f"{pre}.conv1", width, 1)
            y = conv_block(b, y, f"{pre}.conv2", width, 3, stride=s, pad=1)
            y = conv_block(b, y, f"{pre}.conv3", cout, 1, act=None)
            sc = x
            if s != 1 or cin != cout:
                sc = conv_block(b, x, f"{pre}.downsample", cout, 1, stride=s, act=None)
            x = qadd(b, y, sc)
            cin = cout
    return _finish("resnet50", b, _head(b, x), (batch, 3, hw, hw), seed)


def mobilenet_v2(batch: int = 1, seed: int = 4, hw: int = 224) -> Model:
    """Config 5: MobileNetV2 1.0 (stem 3x3/2, 17 inverted residuals, 1x1 1280, fc)."""
    b = _Builder(seed)
    x = _input(b, (batch, 3, hw, hw))
    x = conv_block(b, x, "features.0", 32, 3, stride=2, pad=1, act="relu6")
    cin = 32
    idx = 1
    for t, c, n, s in ((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
                       (6, 320, 1, 1)):
        for i in range(n):
            stride = s if i == 0 else 1
            hidden = cin * t
            pre = f"features.{idx}"
            y = x
            if t != 1:
                y = conv_block(b, y, f"{pre}.expand", hidden, 1, act="relu6")
            y = conv_block(b, y, f"{pre}.dw", hidden, 3, stride=stride, pad=1, groups=hidden, act="relu6")
            y = conv_block(b, y, f"{pre}.project", c, 1, act=None)
            if stride == 1 and cin == c:
                y = qadd(b, y, x, relu=False)
            x = y
            cin = c
            idx += 1
    x = conv_block(b, x, "features.18", 1280, 1, act="relu6")
    return _finish("mobilenet_v2", b, _head(b, x), (batch, 3, hw, hw), seed)


MODELS = {"qnn_dense_128": qnn_dense_128, "lenet5": lenet5, "resnet18": resnet18, "resnet50": resnet50,
          "mobilenet_v2": mobilenet_v2}


def macs_per_sample(model: Model) -> int:
    """Conv + dense multiply-accumulates per sample (BASELINE.md §3 'MAC per sample')."""
    from .relay.build_module import lower
    plan = lower(model.mod, model.params)
    total = 0
    for op in plan.ops:
        if op.op == "qnn.conv2d":
            w = plan.tensor(op.inputs[1])
            o, cg, kh, kw = w.shape
            _, _, oh, ow = op.out.shape
            total += o * oh * ow * cg * kh * kw
        elif op.op == "qnn.dense":
            w = plan.tensor(op.inputs[1])
            total += w.shape[0] * w.shape[1]
    batch = model.input_shape[0]
    return total if model.name == "qnn_dense_128" else total


def trace_bytes_per_sample(model: Model) -> int:
    from .relay.build_module import lower
    plan = lower(model.mod, model.params)
    b = model.input_shape[0]
    return sum(t.nbytes for t in plan.records) // b


# ---------------------------------------------------------------- float32 models (relay.quantize input)

@dataclass
class FloatModel:
    """A float32 graph for ``relay.quantize.quantize``: the reference's
    quantizer consumes float Relay graphs with batch norm already folded (SimplifyInference /
    FoldScaleAxis), i.e. conv -> bias_add -> relu chains."""
    name: str
    mod: relay.IRModule
    params: Dict[str, np.ndarray]
    input_name: str
    input_shape: Tuple[int, ...]
    seed: int

    def random_input(self, seed: Optional[int] = None, batch: Optional[int] = None) -> np.ndarray:
        rng = np.random.default_rng(self.seed + 1000 if seed is None else seed)
        shape = list(self.input_shape)
        if batch is not None:
            shape[0] = batch
        return rng.standard_normal(shape).astype(np.float32)


def resnet_float(depth: int = 18, batch: int = 1, hw: int = 224, seed: int = 5, classes: int = 1000) -> FloatModel:
    """torchvision ResNet-18 / ResNet-50 topology in float32 with He-normal weights and small
    biases (BN folded), seeded; input N(0, 1)."""
    from .relay import op as _op
    rng = np.random.default_rng(seed)
    params: Dict[str, np.ndarray] = {}

    def conv(x, name, cin, cout, k, stride=1, pad=0, relu=True):
        w = relay.var(name + ".weight", (cout, cin, k, k), "float32")
        bvar = relay.var(name + ".bias", (cout,), "float32")
        params[name + ".weight"] = (rng.standard_normal((cout, cin, k, k)) * math.sqrt(2.0 / (cin * k * k))
                                    ).astype(np.float32)
        params[name + ".bias"] = (rng.standard_normal(cout) * 0.05).astype(np.float32)
        y = relay.nn.bias_add(_op.conv2d(x, w, strides=stride, padding=pad), bvar)
        return relay.nn.relu(y) if relu else y

    x = relay.var("data", (batch, 3, hw, hw), "float32")
    y = conv(x, "conv1", 3, 64, 7, 2, 3)
    y = relay.nn.max_pool2d(y, pool_size=(3, 3), strides=(2, 2), padding=(1, 1))
    cin = 64
    stages = ((64, 2, 1), (128, 2, 2), (256, 2, 2), (512, 2, 2)) if depth == 18 else \
        ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))
    for li, (width, blocks, stride) in enumerate(stages):
        cout = width if depth == 18 else width * 4
        for bi in range(blocks):
            s = stride if bi == 0 else 1
            pre = f"layer{li + 1}.{bi}"
            if depth == 18:
                z = conv(y, f"{pre}.conv1", cin, cout, 3, s, 1)
                z = conv(z, f"{pre}.conv2", cout, cout, 3, 1, 1, relu=False)
            else:
                z = conv(y, f"{pre}.conv1", cin, width, 1)
                z = conv(z, f"{pre}.conv2", width, width, 3, s, 1)
                z = conv(z, f"{pre}.conv3", width, cout, 1, relu=False)
            sc = y if (s == 1 and cin == cout) else conv(y, f"{pre}.downsample", cin, cout, 1, s, relu=False)
            y = relay.nn.relu(_op.add(z, sc))
            cin = cout
    y = relay.nn.batch_flatten(relay.nn.global_avg_pool2d(y))
    wf = relay.var("fc.weight", (classes, cin), "float32")
    bf = relay.var("fc.bias", (classes,), "float32")
    params["fc.weight"] = (rng.standard_normal((classes, cin)) / math.sqrt(cin)).astype(np.float32)
    params["fc.bias"] = (rng.standard_normal(classes) * 0.05).astype(np.float32)
    y = relay.nn.bias_add(_op.dense(y, wf), bf)
    return FloatModel(f"resnet{depth}_float", relay.IRModule.from_expr(y), params, "data", (batch, 3, hw, hw), seed)

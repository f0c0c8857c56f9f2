"""Relay-compatible front door: ``relay.var/const``, ``relay.qnn.op.*``, ``relay.nn.*`` and
``relay.build`` (python/tvm/relay/build_module.py:409) targeting the MI355X engine."""
from . import qnn  # noqa: F401
from .expr import (Call, Constant, Expr, Function, IRModule, TensorType, Tuple, Var, const,  # noqa: F401
                   free_vars, post_order, var)
from .op import (add, avg_pool2d, batch_flatten, bias_add, cast, cast_hint, clip, fixed_point_multiply,  # noqa: F401
                 global_avg_pool2d, left_shift, max_pool2d, multiply, relu, reshape, right_shift, round, stop_fusion,
                 transpose)
from . import op as _op
from .parser import ParseError, astext, fromtext, parse  # noqa: F401  (tvm.parser.parse / fromtext)
from . import contrib  # noqa: F401,E402  (relay.op.contrib.tachikoma analogue: contrib.tachikoma)
from . import quantize  # noqa: F401,E402  (relay.quantize: float32 graph -> integer graph)
from . import transform  # noqa: F401,E402  (relay.transform: SimplifyInference, FoldScaleAxis, FoldConstant)


class _NN:
    bias_add = staticmethod(_op.bias_add)
    relu = staticmethod(_op.relu)
    max_pool2d = staticmethod(_op.max_pool2d)
    avg_pool2d = staticmethod(_op.avg_pool2d)
    global_avg_pool2d = staticmethod(_op.global_avg_pool2d)
    batch_flatten = staticmethod(_op.batch_flatten)
    conv2d = staticmethod(_op.conv2d)
    dense = staticmethod(_op.dense)
    batch_norm = staticmethod(_op.batch_norm)
    pad = staticmethod(_op.pad)


nn = _NN()


class analysis:  # noqa: N801  (mirrors relay.analysis)
    free_vars = staticmethod(free_vars)
    post_order = staticmethod(post_order)


def save_param_dict(params):
    """relay.save_param_dict (python/tvm/relay/param_dict.py) → runtime.save_param_dict."""
    from ..runtime import save_param_dict as _s
    return _s(params)


def load_param_dict(param_bytes):
    from ..runtime import load_param_dict as _l
    return _l(param_bytes)


def build(mod, target: str = "mi355x", params=None, mod_name: str = "default", fuse: bool = True):
    """``relay.build``: lower a QNN module to the MI355X engine (see build_module.py).

    ``fuse=False`` keeps one device kernel per Relay op (the literal per-op record-and-run
    shape); the default fuses conv/dense layer blocks, writing the same records."""
    from .build_module import build as _build
    return _build(mod, target=target, params=params, mod_name=mod_name, fuse=fuse)

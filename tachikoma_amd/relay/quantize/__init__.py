"""``relay.quantize``: float32 graph -> integer-only graph.

Reference: python/tvm/relay/quantize/quantize.py (qconfig :37-216, quantize :330-379),
_partition.py, _annotate.py, _calibrate.py (:158-238), src/relay/quantize/realize.cc.
``quantize(mod, params)`` runs the same pipeline — prerequisite optimisation, partition,
annotate, calibrate, realize, FoldConstant — over this package's IR; the result is an
ordinary graph of ``nn.conv2d`` (int8 x int8 -> int32), ``add``, ``right_shift``, ``clip``,
``cast`` ... that ``relay.build`` runs and traces on the MI355X like any other graph.
"""
from .qconfig import QAnnotateKind, QConfig, current_qconfig, qconfig  # noqa: F401
from .passes import (annotate, calibrate, partition, prerequisite_optimize, quantize,  # noqa: F401
                     realize, simulated_quantize)

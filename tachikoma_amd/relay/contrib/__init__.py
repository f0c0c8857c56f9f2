"""``relay.op.contrib`` analogue: operator-offload (BYOC) partitioners for the MI355X engine."""
from . import tachikoma  # noqa: F401

"""Debug executor (python/tvm/contrib/debugger analogue)."""
from . import debug_executor  # noqa: F401

from . import graph_executor  # noqa: F401

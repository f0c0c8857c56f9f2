from . import op  # noqa: F401

from . import _wrapper  # noqa: F401

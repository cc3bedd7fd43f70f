from .model import MapAnything  # noqa: F401

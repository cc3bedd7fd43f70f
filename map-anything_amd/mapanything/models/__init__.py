"""Model factory surface (reference mapanything/models/__init__.py:18-22)."""

from .mapanything import MapAnything  # noqa: F401

__all__ = ["MapAnything"]

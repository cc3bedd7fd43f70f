from .base import MultiViewTransformerInput, MultiViewTransformerOutput  # noqa: F401

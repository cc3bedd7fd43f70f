"""Info-sharing I/O dataclasses (uniception/models/info_sharing/base.py:75-91)."""
from dataclasses import dataclass
from typing import List, Optional

from torch import Tensor


@dataclass
class MultiViewTransformerInput:
    features: List[Tensor]                          # per view (B, input_embed_dim, h, w)
    additional_input_tokens: Optional[Tensor] = None  # (B, input_embed_dim, num_additional_tokens)


@dataclass
class MultiViewTransformerOutput:
    features: List[Tensor]                            # per view (B, transformer_embed_dim, h, w)
    additional_token_features: Optional[Tensor] = None  # (B, transformer_embed_dim, num_additional_tokens)

"""DPT hand-off dataclass (uniception/models/prediction_heads/dpt.py:24-26)."""
from dataclasses import dataclass
from typing import Tuple

from torch import Tensor


@dataclass
class DPTFeatureInput:
    features_upsampled_8x: Tensor  # (B, 256, 8h, 8w)
    target_output_shape: Tuple[int, int]

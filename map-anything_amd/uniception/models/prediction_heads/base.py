"""Prediction-head / adaptor I/O dataclasses (uniception/models/prediction_heads/base.py:14-103)."""
from dataclasses import dataclass
from typing import List, Tuple

from torch import Tensor


@dataclass
class PredictionHeadInput:
    last_feature: Tensor  # (B, C, h, w)


@dataclass
class PredictionHeadLayeredInput:
    list_features: List[Tensor]  # each (B, C_i, h, w)
    target_output_shape: Tuple[int, int]


@dataclass
class PredictionHeadTokenInput:
    last_feature: Tensor  # (B, C, T)


@dataclass
class PixelTaskOutput:
    decoded_channels: Tensor  # (B, C, H, W)


@dataclass
class SummaryTaskOutput:
    decoded_channels: Tensor  # (B, C)


@dataclass
class AdaptorInput:
    adaptor_feature: Tensor
    output_shape_hw: Tuple[int, int]


@dataclass
class AdaptorOutput:
    value: Tensor


@dataclass
class MaskAdaptorOutput:
    logits: Tensor  # (B, 1, H, W)
    mask: Tensor    # (B, 1, H, W)


@dataclass
class RegressionWithConfidenceAndMaskAdaptorOutput:
    value: Tensor       # (B, C, H, W)
    confidence: Tensor  # (B, 1, H, W)
    logits: Tensor      # (B, 1, H, W)
    mask: Tensor        # (B, 1, H, W)

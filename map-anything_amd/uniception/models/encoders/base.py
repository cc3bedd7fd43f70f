"""Encoder I/O dataclasses (uniception/models/encoders/base.py:14-117)."""
from dataclasses import dataclass

from torch import Tensor


@dataclass
class EncoderInput:
    data_norm_type: str


@dataclass
class EncoderOutput:
    pass


@dataclass
class EncoderGlobalRepInput:
    data: Tensor  # (B, C)


@dataclass
class EncoderGlobalRepOutput:
    features: Tensor  # (B, enc_embed_dim)


@dataclass
class ViTEncoderInput(EncoderInput):
    image: Tensor  # (B, 3, H, W), normalised as data_norm_type says


@dataclass
class ViTEncoderNonImageInput:
    data: Tensor  # (B, C, H, W)


@dataclass
class ViTEncoderOutput(EncoderOutput):
    features: Tensor  # (B, enc_embed_dim, H / patch, W / patch)

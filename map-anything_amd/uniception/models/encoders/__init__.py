from .base import (EncoderGlobalRepInput, EncoderGlobalRepOutput, EncoderInput, EncoderOutput,  # noqa: F401
                   ViTEncoderInput, ViTEncoderNonImageInput, ViTEncoderOutput)

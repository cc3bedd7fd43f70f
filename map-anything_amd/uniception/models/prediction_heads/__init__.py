from .base import (AdaptorInput, AdaptorOutput, MaskAdaptorOutput, PixelTaskOutput,  # noqa: F401
                   PredictionHeadInput, PredictionHeadLayeredInput, PredictionHeadTokenInput,
                   RegressionWithConfidenceAndMaskAdaptorOutput, SummaryTaskOutput)
from .dpt import DPTFeatureInput  # noqa: F401

"""Module-level operator surface of the MapAnything path (second row): the reference model calls
its sub-modules with uniception dataclasses (model.py:670-767, 1440-1655), e.g.

    enc = model.encoder(ViTEncoderInput(image=img, data_norm_type="dinov2")).features        # (B, 1024, h, w)
    final, inter = model.info_sharing(MultiViewTransformerInput(features=[...], additional_input_tokens=tok))
    dense = model.dense_head(PredictionHeadLayeredInput(list_features=[...], target_output_shape=(H, W)))
    out = model.dense_adaptor(AdaptorInput(adaptor_feature=dense.decoded_channels, output_shape_hw=(H, W)))

These classes keep those names, inputs and outputs and run the engine's HIP stages (engine.py) on the model's
device in the model's precision.  Inputs and outputs are the reference's channel-first layouts (fp32); the engine
works token-major (rows = pixels, channels contiguous), so each module converts at its boundary (a permute copy)
— the per-view forward itself (MapAnything.forward / infer) never goes through here.  Dataclasses are read by
attribute name, so the reference's own uniception instances are accepted as well.  Batch elements (B > 1) are
independent multi-view sets and are run one after another (the engine carries one view set per call).
"""
from __future__ import annotations

from typing import List

import torch

from uniception.models.encoders import ViTEncoderOutput
from uniception.models.info_sharing import MultiViewTransformerOutput
from uniception.models.prediction_heads import (AdaptorOutput, DPTFeatureInput, PixelTaskOutput,
                                                RegressionWithConfidenceAndMaskAdaptorOutput, SummaryTaskOutput)

from ... import _native as nat
from .engine import ENC_DIM, PATCH

f32 = torch.float32


def _rows(x: torch.Tensor, dtype) -> torch.Tensor:
    """(B, C, h, w) -> token rows [B*h*w][C] in the engine's dtype (layout copy at the module boundary)."""
    B, C, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(B * h * w, C).to(dtype).contiguous()


def _chw(rows: torch.Tensor, B: int, h: int, w: int) -> torch.Tensor:
    """token rows [B*h*w][C] -> (B, C, h, w) fp32."""
    return rows.reshape(B, h, w, -1).permute(0, 3, 1, 2).to(f32).contiguous()


class _EngineModule:
    def __init__(self, model):
        self._model = model

    def _eng(self):
        return self._model.engine()

    def __call__(self, *args, **kwargs):
        return self.forward(*args, **kwargs)

    def _dev(self, t: torch.Tensor, dtype=f32) -> torch.Tensor:
        return t.to(self._model.device, dtype)


class DINOv2Encoder(_EngineModule):
    """uniception/models/encoders/dinov2.py:146-178 (ViT-L/14, final norm, cls dropped)."""
    data_norm_type = "dinov2"
    enc_embed_dim = ENC_DIM
    patch_size = PATCH

    @torch.no_grad()
    def forward(self, encoder_input) -> ViTEncoderOutput:
        if encoder_input.data_norm_type != self.data_norm_type:
            raise AssertionError(f"Input data norm type {encoder_input.data_norm_type} does not match encoder norm "
                                 f"type {self.data_norm_type}")
        img = self._dev(encoder_input.image).contiguous()
        B, _, H, W = img.shape
        if H % PATCH or W % PATCH:
            raise AssertionError(f"Input shape must be divisible by patch size: {PATCH}")
        eng = self._eng()
        with torch.cuda.device(eng.device):
            enc = eng.encoder_features(img)
            nat.check_faults()  # the LayerNorm-fused residual linears' band barriers (include/mapa.h fault channel)
        return ViTEncoderOutput(features=_chw(enc, B, H // PATCH, W // PATCH))


class MultiViewAlternatingAttentionTransformerIFR(_EngineModule):
    """uniception/models/info_sharing/alternating_attention_transformer.py:530-771 (released config: depth 24,
    dim 768, IFR indices [11, 17], intermediates normed; any depth / width with 64-wide heads / 2 or 3 indices,
    e.g. the 48-layer width-1024 configs) — or, for a global_attention config, the GAT of
    global_attention_transformer.py:458-640 (the engine follows model.info).  Exactly one additional input token
    (MapAnything's scale token)."""
    @property
    def dim(self):
        return self._model.info.dim

    @property
    def indices(self):
        return self._model.info.indices

    @torch.no_grad()
    def forward(self, model_input):
        feats: List[torch.Tensor] = list(model_input.features)
        tok = model_input.additional_input_tokens
        if tok is None or tok.dim() != 3 or tok.shape[-1] != 1 or tok.shape[1] != ENC_DIM:
            raise NotImplementedError("this engine's info-sharing module takes exactly one additional token "
                                      "(B, 1024, 1) — MapAnything's scale token")
        V = len(feats)
        B, C, h, w = feats[0].shape
        if C != ENC_DIM or any(f.shape != feats[0].shape for f in feats):
            raise AssertionError("every view's features must be (B, 1024, h, w)")
        T = h * w
        eng = self._eng()
        idx, D = self._model.info.indices, self._model.info.dim
        final, final_tok = [None] * B, [None] * B
        inter = [[None] * B for _ in idx]
        inter_tok = [[None] * B for _ in idx]
        with torch.cuda.device(eng.device):
            for b in range(B):
                f32 = torch.empty(V * T + 1, ENC_DIM, dtype=torch.float32, device=eng.device)
                f32[:V * T] = _rows(torch.stack([self._dev(f[b]) for f in feats], 0), torch.float32)
                f32[V * T] = self._dev(tok[b, :, 0], torch.float32)
                taps = {}
                eng.aat(f32.to(eng.lp), V, T, taps, pe_idx=self._model._view_pe_rows(V), fused_f32=f32)
                final[b], final_tok[b] = taps["aat_final"].reshape(V, h, w, D), taps["scale_token"]
                for j, d in enumerate(idx):
                    inter[j][b] = taps[f"aat_l{d}"].reshape(V, h, w, D)
                    inter_tok[j][b] = taps[f"aat_l{d}_token"]
            nat.check_faults()

        def pack(per_b, toks):
            views = [torch.stack([per_b[b][v] for b in range(B)], 0).permute(0, 3, 1, 2).contiguous()
                     for v in range(V)]
            return MultiViewTransformerOutput(features=views,
                                              additional_token_features=torch.stack(
                                                  [t.reshape(D, 1) for t in toks], 0))

        return pack(final, final_tok), [pack(inter[j], inter_tok[j]) for j in range(len(idx))]


MultiViewGlobalAttentionTransformerIFR = MultiViewAlternatingAttentionTransformerIFR  # same engine entry


class DPTFeature(_EngineModule):
    """uniception/models/prediction_heads/dpt.py:180-232: four features (1024, 768, 768, 768 channels; with three
    info-sharing taps all four are the transformer's width, model.py:362-372) -> the
    256-channel map at 8x the token grid."""

    @torch.no_grad()
    def forward(self, head_input) -> DPTFeatureInput:
        f0, f1, f2, f3 = head_input.list_features
        B, _, h, w = f0.shape
        eng = self._eng()
        with torch.cuda.device(eng.device):
            rows = [eng.head_rows(_rows(self._dev(f), f32)) for f in (f0, f1, f2, f3)]
            _, feat = eng.dpt_feature(rows[0], rows[1], rows[2], rows[3], B, h, w, want_f32=True)
        return DPTFeatureInput(features_upsampled_8x=feat.permute(0, 3, 1, 2).contiguous(),
                               target_output_shape=tuple(head_input.target_output_shape))


class DPTRegressionProcessor(_EngineModule):
    """uniception/models/prediction_heads/dpt.py:285-311: conv3x3 -> bilinear (align_corners) to the target
    shape -> conv3x3 + ReLU -> conv1x1 to 6 channels (raw, before the adaptor)."""

    def __init__(self, model):
        super().__init__(model)
        self._w6 = {}

    @torch.no_grad()
    def forward(self, dpt_input) -> PixelTaskOutput:
        x = dpt_input.features_upsampled_8x
        H, W = (int(v) for v in dpt_input.target_output_shape)
        B, _, hf, wf = x.shape
        eng = self._eng()
        with torch.cuda.device(eng.device):
            hid = eng.dpt_regress(eng.head_rows(_rows(self._dev(x), f32)), B, hf, wf, H, W)
            w6 = self._w6.get(hid.dtype)
            if w6 is None:
                w6 = self._w6[hid.dtype] = torch.empty(6, 128, dtype=hid.dtype, device=eng.device)
                nat.convert_rows(eng.w.reg_w6, 128, 6, 128, w6, 128)
            raw = torch.empty(B * H * W, 6, dtype=f32, device=eng.device)
            nat.gemm(hid, w6, B * H * W, 6, 128, bias=eng.w.reg_b6, out_f32=raw)
        return PixelTaskOutput(decoded_channels=_chw(raw, B, H, W))


class DenseHead:
    """nn.Sequential(dpt_feature_head, dpt_regressor_head) (model.py:394-399)."""

    def __init__(self, feature_head: DPTFeature, regressor_head: DPTRegressionProcessor):
        self.feature_head, self.regressor_head = feature_head, regressor_head

    def __call__(self, head_input) -> PixelTaskOutput:
        return self.regressor_head(self.feature_head(head_input))

    forward = __call__


class RayDirectionsPlusDepthWithConfidenceAndMaskAdaptor(_EngineModule):
    """adaptors.py:1898-1951: 6 raw channels -> value (unit ray directions (3) + exp depth (1)), confidence
    (1 + exp), mask logits and sigmoid mask."""

    @torch.no_grad()
    def forward(self, adaptor_input) -> RegressionWithConfidenceAndMaskAdaptorOutput:
        x = adaptor_input.adaptor_feature
        B, C, H, W = x.shape
        if C != 6:
            raise AssertionError(f"dense adaptor expects 6 channels, got {C}")
        eng = self._eng()
        dev = eng.device
        with torch.cuda.device(dev):
            raw = _rows(self._dev(x), f32)
            value = torch.empty(B, 4, H, W, dtype=f32, device=dev)
            conf, logits, mask = (torch.empty(B, 1, H, W, dtype=f32, device=dev) for _ in range(3))
            nat.dense_adaptor(raw, B, H * W, value, conf, logits, mask)
        return RegressionWithConfidenceAndMaskAdaptorOutput(value=value, confidence=conf, logits=logits, mask=mask)


class PoseHead(_EngineModule):
    """uniception/models/prediction_heads/pose_head.py:50-159: (B, 768, h, w) -> (B, 7) raw."""

    @torch.no_grad()
    def forward(self, head_input) -> SummaryTaskOutput:
        x = head_input.last_feature
        B, _, h, w = x.shape
        eng = self._eng()
        with torch.cuda.device(eng.device):
            raw = eng.pose(eng.head_rows(_rows(self._dev(x), f32)), B, h * w)
        return SummaryTaskOutput(decoded_channels=raw)


class CamTranslationPlusQuatsAdaptor(_EngineModule):
    """adaptors.py:688-732: (B, 7) raw -> cat(translation, unit quaternion)."""

    @torch.no_grad()
    def forward(self, adaptor_input) -> AdaptorOutput:
        raw = self._dev(adaptor_input.adaptor_feature).reshape(-1, 7).contiguous()
        B = raw.shape[0]
        dev = raw.device
        with torch.cuda.device(dev):
            pose_out = torch.empty(B, 19, dtype=f32, device=dev)
            scale = torch.empty(1, dtype=f32, device=dev)
            nat.pose_scale_finalize(raw, torch.zeros(1, dtype=f32, device=dev), B, 1, pose_out, scale, None)
        return AdaptorOutput(value=torch.cat([pose_out[:, 16:19], pose_out[:, 3:7]], 1))


class MLPHead(_EngineModule):
    """uniception/models/prediction_heads/mlp_head.py:13-92 on the scale token: (B, 768, 1) -> (B, 1, 1)."""

    @torch.no_grad()
    def forward(self, head_input) -> SummaryTaskOutput:
        x = self._dev(head_input.last_feature)
        D = self._model.info.dim
        if x.dim() != 3 or x.shape[1] != D or x.shape[2] != 1:
            raise AssertionError(f"scale head expects (B, {D}, 1), got {tuple(x.shape)}")
        eng = self._eng()
        with torch.cuda.device(eng.device):
            out = torch.stack([eng.scale(x[b, :, 0].reshape(1, D).contiguous()) for b in range(x.shape[0])])
        return SummaryTaskOutput(decoded_channels=out.reshape(-1, 1, 1))


class ScaleAdaptor(_EngineModule):
    """adaptors.py:171-212 (mode exp, bounds [1e-8, inf])."""

    @torch.no_grad()
    def forward(self, adaptor_input) -> AdaptorOutput:
        x = self._dev(adaptor_input.adaptor_feature)
        B = x.shape[0]
        dev = x.device
        with torch.cuda.device(dev):
            pose_out = torch.empty(B, 19, dtype=f32, device=dev)
            scale = torch.empty(B, dtype=f32, device=dev)
            dummy_pose = torch.zeros(B, 7, dtype=f32, device=dev)
            dummy_pose[:, 6] = 1.0
            nat.pose_scale_finalize(dummy_pose, x.reshape(B).contiguous(), B, B, pose_out, scale, None)
        return AdaptorOutput(value=scale.reshape(x.shape))


class FusionNorm(_EngineModule):
    """fusion_norm_layer = nn.LayerNorm(1024, eps 1e-6) (model.py:213), applied channel-last (model.py:1424-1432):
    x (..., 1024) fp32 -> same shape fp32."""

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if x.shape[-1] != ENC_DIM:
            raise AssertionError(f"fusion norm expects (..., {ENC_DIM}), got {tuple(x.shape)}")
        eng = self._eng()
        src = self._dev(x).reshape(-1, ENC_DIM).contiguous()
        out = torch.empty_like(src)
        with torch.cuda.device(eng.device):
            eng._ln(src, src.shape[0], ENC_DIM, eng.w.fus_w, eng.w.fus_b, y_f32=out)
        return out.reshape(x.shape)

    forward = __call__

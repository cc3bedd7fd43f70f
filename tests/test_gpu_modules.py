"""Module-level API (uniception dataclass contracts): the reference's own module chain
(model.py:670-767 encoder, 1292-1438 fusion, 530-771 info sharing, 1440-1655 heads + adaptors) rebuilt from the
engine's modules reproduces the reference's stage taps and outputs (fixtures from the real reference)."""

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2
from tests_helpers import CASES, make_views

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model32():
    from mapanything.models import MapAnything
    from tests_helpers import released_config

    return MapAnything(**released_config(), precision="fp32").load_synthetic_weights().to("cuda").eval()


def _chain(model, views):
    from uniception.models.encoders import ViTEncoderInput
    from uniception.models.info_sharing import MultiViewTransformerInput
    from uniception.models.prediction_heads import (AdaptorInput, PredictionHeadInput, PredictionHeadLayeredInput,
                                                    PredictionHeadTokenInput)

    imgs = [v["img"].cuda() for v in views]
    H, W = imgs[0].shape[-2:]
    enc = [model.encoder(ViTEncoderInput(image=i, data_norm_type="dinov2")).features for i in imgs]
    fused = [model.fusion_norm_layer(e.permute(0, 2, 3, 1)).permute(0, 3, 1, 2) for e in enc]
    tok = model.scale_token.reshape(1, -1, 1)
    final, inter = model.info_sharing(MultiViewTransformerInput(features=fused, additional_input_tokens=tok))
    cat = lambda xs: torch.cat(xs, 0)  # noqa: E731  views along the batch dim for the heads (model.py:1800-1830)
    layered = PredictionHeadLayeredInput(list_features=[cat(fused), cat(inter[0].features), cat(inter[1].features),
                                                        cat(final.features)], target_output_shape=(H, W))
    dpt = model.dpt_feature_head(layered)
    dense = model.dpt_regressor_head(dpt)
    dense_out = model.dense_adaptor(AdaptorInput(adaptor_feature=dense.decoded_channels, output_shape_hw=(H, W)))
    pose_raw = model.pose_head(PredictionHeadInput(last_feature=cat(final.features))).decoded_channels
    pose = model.pose_adaptor(AdaptorInput(adaptor_feature=pose_raw, output_shape_hw=(H, W))).value
    scale_raw = model.scale_head(PredictionHeadTokenInput(last_feature=final.additional_token_features))
    scale = model.scale_adaptor(AdaptorInput(adaptor_feature=scale_raw.decoded_channels, output_shape_hw=(H, W)))
    return dict(enc=enc, fused=fused, final=final, inter=inter, dpt=dpt, dense=dense, dense_out=dense_out,
                pose_raw=pose_raw, pose=pose, scale_raw=scale_raw.decoded_channels, scale=scale.value,
                dense_seq=model.dense_head(layered))


def test_module_chain_matches_reference_taps(model32, golden):
    name = "cfg1_224"
    g = golden(name)
    _, ts, ds = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))[name]["steps_out_tap_dpt"]
    views = make_views(CASES[name])
    c = _chain(model32, views)
    npy = lambda t: t.detach().float().cpu().numpy()  # noqa: E731
    assert rel_l2(npy(torch.cat(c["enc"], 0))[:, :, ::ts, ::ts], g["tap_encoder"]) < 1e-4
    fused_nhwc = npy(torch.cat(c["fused"], 0).permute(0, 2, 3, 1))
    assert rel_l2(fused_nhwc[:, ::ts, ::ts], g["tap_fused_nhwc"]) < 1e-4
    for key, out in (("tap_aat_final", c["final"]), ("tap_aat_l11", c["inter"][0]), ("tap_aat_l17", c["inter"][1])):
        mine = npy(torch.stack(out.features, 1))[..., ::ts, ::ts]
        assert rel_l2(mine, g[key]) < 1e-4, key
    assert rel_l2(npy(c["final"].additional_token_features), g["tap_scale_token"]) < 1e-4
    assert rel_l2(npy(c["dpt"].features_upsampled_8x)[:, :, ::ds, ::ds], g["tap_dpt_feature"]) < 1e-4
    assert rel_l2(npy(c["pose_raw"]), g["tap_pose_raw"]) < 1e-4
    assert rel_l2(npy(c["scale_raw"]), g["tap_scale_raw"]) < 1e-4
    # adaptors -> the reference's final outputs (model.py:1871-1923: depth and translation carry the metric scale)
    step = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))[name]["steps_out_tap_dpt"][0]
    val = c["dense_out"].value
    rays = npy(val[:, 0:3].permute(0, 2, 3, 1))[:, ::step, ::step]
    assert rel_l2(rays, g["out_ray_directions"][:, 0]) < 1e-4
    s = c["scale"].reshape(-1)[0]
    depth = npy((val[:, 3:4] * s).permute(0, 2, 3, 1))[:, ::step, ::step]
    assert rel_l2(depth, g["out_depth_along_ray"][:, 0]) < 1e-4
    assert rel_l2(npy(c["dense_out"].confidence[:, 0])[:, ::step, ::step], g["out_conf"][:, 0]) < 1e-4
    logits = npy(c["dense_out"].logits[:, 0])[:, ::step, ::step]
    assert rel_l2(logits, g["out_non_ambiguous_mask_logits"][:, 0]) < 1e-4
    assert rel_l2(npy(c["scale"]).reshape(1), g["out_metric_scaling_factor"][0].reshape(1)) < 1e-4
    assert rel_l2(npy(c["pose"][:, 3:7]), g["out_cam_quats"][:, 0]) < 1e-4
    assert rel_l2(npy(c["pose"][:, 0:3] * s), g["out_cam_trans"][:, 0]) < 1e-4
    # nn.Sequential(dpt_feature_head, dpt_regressor_head) is the same computation
    assert torch.equal(c["dense_seq"].decoded_channels, c["dense"].decoded_channels)
    # the adaptor's mask is the sigmoid probability; the model output thresholds it at 0.5
    assert torch.allclose(c["dense_out"].mask, torch.sigmoid(c["dense_out"].logits), atol=1e-6)


def test_module_chain_equals_forward_bf16():
    """bf16 model: the module chain and MapAnything.forward produce the same predictions within bf16 noise."""
    from mapanything.models import MapAnything
    from tests_helpers import released_config

    m = MapAnything(**released_config()).load_synthetic_weights().to("cuda").eval()
    views = make_views(CASES["cfg1_224"])
    c = _chain(m, views)
    fw = m.forward([{**v, "img": v["img"].cuda()} for v in views])
    rays = torch.cat([p["ray_directions"] for p in fw], 0)
    mine = c["dense_out"].value[:, 0:3].permute(0, 2, 3, 1)
    assert rel_l2(mine.cpu().numpy(), rays.cpu().numpy()) < 2e-2
    s_mine, s_fw = c["scale"].reshape(-1)[0].item(), fw[0]["metric_scaling_factor"].item()
    assert rel_l2(np.array([s_mine]), np.array([s_fw])) < 2e-2


def test_module_input_contracts(model32):
    from uniception.models.encoders import ViTEncoderInput
    from uniception.models.info_sharing import MultiViewTransformerInput

    img = torch.zeros(1, 3, 224, 224, device="cuda")
    with pytest.raises(AssertionError):
        model32.encoder(ViTEncoderInput(image=img, data_norm_type="identity"))
    with pytest.raises(AssertionError):
        model32.encoder(ViTEncoderInput(image=img[..., :220], data_norm_type="dinov2"))
    f = torch.zeros(1, 1024, 4, 4, device="cuda")
    with pytest.raises(NotImplementedError):
        model32.info_sharing(MultiViewTransformerInput(features=[f, f]))

"""Range safety of the default TF32-equivalent heads (head_precision "tf32": binary16 operands at TF32's 11
significant bits).  TF32 keeps fp32's 8-bit exponent (the reference's fp32 heads on its GPUs, model.py:89-93 /
1774); binary16 has 5 bits.  The engine closes that gap two ways:
  * weights: a head weight whose largest magnitude lies outside [2^-4, 2^12] is stored as 2^s x w and the GEMM
    epilogue takes the power of two back out exactly (engine._f16_wscale, _native._wscale_epilogue), so tiny weights
    keep their 11 bits as TF32 keeps them;
  * activations: one that leaves binary16's range sets MAPA_FAULT_F16_RANGE and infer() / forward() re-run the call
    with the fp32-exact heads (MapAnything._range_fallback) instead of raising.
"""

import numpy as np
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu

from tests_helpers import CASES, make_views, released_config

TF32_BOUND = 3e-3  # test_gpu_model.HEAD_BOUND["tf32"]
HEAD_PREFIXES = ("dpt_feature_head.", "dpt_regressor_head.", "pose_head.")


def _scaled_sd(factor):
    """The synthetic checkpoint with every head conv / linear WEIGHT (not the biases) multiplied by factor."""
    from mapanything.models.mapanything.spec import canonical_spec
    from mapanything.utils.synthetic import synthetic_state_dict

    sd = synthetic_state_dict(canonical_spec())
    out = {}
    for k, v in sd.items():
        v = np.asarray(v, np.float32)
        if k.startswith(HEAD_PREFIXES) and k.endswith(".weight") and v.ndim >= 2:
            v = v * np.float32(factor)
        out[k] = torch.from_numpy(np.ascontiguousarray(v))
    return out


def _model(sd, **kw):
    from mapanything.models import MapAnything

    return MapAnything(**released_config(), **kw).load_state_dict(sd).to("cuda").eval()


def _same(a, b):
    """Bitwise equal, NaN positions included."""
    a, b = a.float(), b.float()
    return torch.equal(torch.isnan(a), torch.isnan(b)) and torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))


@pytest.mark.parametrize("graphs", [False, True])
def test_overflow_head_weights_x300_fall_back_to_fp32_exact_heads(graphs):
    """Head weights x300: the activations outgrow binary16 (>65504) within two layers; infer() returns exactly what the
    fp32-exact heads return on the same weights (head_precision='fp32'), eager and graph-replayed, instead of raising."""
    from mapanything import _native as nat
    from mapanything.models import MapAnything

    sd = _scaled_sd(300.0)
    views = make_views(CASES["cfg1_224"])
    kw = dict(use_amp=True, apply_mask=False)
    m = _model(sd, hip_graphs=graphs)
    assert m.engine("bf16").hfmt == "f16"
    ref = _model(sd, hip_graphs=graphs, head_precision="fp32").infer(views, **kw)
    n0 = MapAnything.range_fallbacks
    with pytest.warns(UserWarning) if n0 == 0 else _null():
        out = m.infer(views, **kw)
    assert MapAnything.range_fallbacks == n0 + 1
    assert nat.fault_status(reset=False) == 0
    for a, b in zip(out, ref):
        for k in ("pts3d", "depth_along_ray", "conf", "cam_trans", "cam_quats", "metric_scaling_factor"):
            assert _same(a[k], b[k]), k
    # forward() takes the same fallback
    n1 = MapAnything.range_fallbacks
    m.forward(_preprocess(make_views(CASES["cfg1_224"])))
    assert MapAnything.range_fallbacks == n1 + 1


def _preprocess(views):
    from mapanything.utils.inference import preprocess_input_views_for_inference, validate_input_views_for_inference

    v = validate_input_views_for_inference(views)
    for x in v:
        for k in list(x.keys()):
            if isinstance(x[k], torch.Tensor):
                x[k] = x[k].cuda()
    return preprocess_input_views_for_inference(v)


def _null():
    import contextlib

    return contextlib.nullcontext()


def test_underflow_head_weights_x1e3_keep_the_tf32_bound():
    """Head weights x1e-3 (most elements below binary16's normal range, 2^-14): stored with a power-of-two scale they
    keep TF32's 11 bits, so the TF32-equivalent heads stay within the tf32 bound of the fp32-exact heads on identical
    fp32 inputs (the stage-level comparison of test_split_precision_heads_match_fp32_heads_at_cfg2_size), with no
    fault and no fallback."""
    from mapanything import _native as nat

    sd = _scaled_sd(1e-3)
    m = _model(sd)
    e32, e16 = m.engine("fp32"), m.engine("bf16")
    assert e16.hfmt == "f16"
    scaled = [t for t in (e16.w.reg_c1, e16.w.reg_c2, e16.w.layer_rn[0], e16.w.pose_proj)
              if getattr(t, "_mapa_wscale", 0)]
    assert len(scaled) == 4, "every head weight x1e-3 is stored with a power-of-two scale"
    case = CASES["cfg1_224"]
    imgs = torch.cat([v["img"] for v in make_views(case)], 0).cuda()
    V, H, W = case["views"], case["h"], case["w"]
    hp, wp = H // 14, W // 14
    taps = {}
    e32.run(imgs, taps=taps)
    tok = taps["scale_token"].view(1, -1).contiguous()
    fin = torch.cat([taps["aat_final"], tok], 0).contiguous()
    nat.fault_status(reset=True)
    res = {}
    for name, eng in (("fp32", e32), ("tf32", e16)):
        t2 = {}
        out = eng.run_heads(eng.head_rows(taps["fused"].contiguous()), eng.head_rows(taps["aat_l11"].contiguous()),
                            eng.head_rows(taps["aat_l17"].contiguous()), eng.head_rows(fin), tok, V, hp, wp, H, W,
                            taps=t2)
        torch.cuda.synchronize()
        res[name] = dict(out, pose_raw=t2["pose_raw"], dpt_feature=t2["dpt_feature"])
    assert nat.fault_status(reset=True) == 0
    bad = {}
    print("\n[tf32 heads vs fp32 heads, head weights x1e-3] rel-L2:")
    for k in ("dpt_feature", "pts3d", "depth_along_ray", "conf", "non_ambiguous_mask_logits", "pose_raw", "cam_trans",
              "cam_quats"):
        e = rel_l2(res["tf32"][k].float().cpu().numpy(), res["fp32"][k].float().cpu().numpy())
        print(f"  {k:28s} {e:.3e}")
        if not e <= TF32_BOUND:
            bad[k] = e
    assert not bad, bad


def test_weight_scale_is_exact_on_normal_weights():
    """The power-of-two storage scale changes no output bit where it is not needed: a weight forced to a scale of
    2^5 (storage 32 x w, epilogue bias x 32, gamma 2^-5) gives the same outputs as the unscaled weight."""
    from mapanything import _native as nat

    torch.manual_seed(0)
    M, N, K = 1000, 96, 256
    A = (torch.randn(M, K, device="cuda") * 0.5).half()
    # magnitudes in [0.01, 0.1]: normal binary16 numbers both as w and as 32 w (the scale is exact there; below
    # 2^-14 the scaled copy keeps bits the unscaled one loses — the point of the scale)
    w = torch.sign(torch.randn(N, K, device="cuda")) * (0.01 + 0.09 * torch.rand(N, K, device="cuda"))
    b = torch.randn(N, device="cuda")
    W0 = w.half()
    W0._mapa_split = True
    W1 = (w * 32).half()
    W1._mapa_split = True
    W1._mapa_wscale = 5
    outs = []
    for Wt in (W0, W1):
        o = torch.empty(M, N, device="cuda")
        r = torch.empty(M, N, device="cuda", dtype=torch.float16)
        nat.gemm(A, Wt, M, N, K, bias=b, act=nat.ACT_RELU, out_f32=o, out_lp_relu=r)
        outs.append((o, r))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])

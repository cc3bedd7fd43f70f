"""Generate the committed golden fixtures from the REAL reference (run in the build container only).

    python tests/golden/make_golden.py          # writes tests/golden/*.npz + *.json

The reference (/root/reference) is imported through `ref_harness.py`, loaded with the
named-PRNG synthetic checkpoint of `mapanything/utils/synthetic.py`, and run through its own
`MapAnything.infer` (model.py:2206-2355, apply_mask=False) on seeded inputs.  What is saved is data only:
inputs are regenerated from their seeds by the same generator, outputs and per-stage taps are stored as
float32 arrays.  Nothing here travels to the GPU box except these fixture files.

Cases:
  cfg1_224   2 views 224x224 image-only, fp32 (full outputs + taps)
  v2_518     2 views 518x518 image-only, fp32 (outputs subsampled [::7, ::7] + taps subsampled)
  mm_224     2 views 224x224 + intrinsics + 90 %-sparse depth_z + is_metric_scale (full outputs + taps)
  cfg2_518   configs[1] itself: 8 views 518x518 image-only, the bench's input seed (outputs [::7, ::7], taps strided)
  cfg4_518   configs[3] itself: 32 views 518x518 + intrinsics + 90 %-sparse depth_z + is_metric_scale (its bf16
             yardstick and spread come from make_yardstick_spread.py)
  b2_224     3 views 224x224 with TWO scenes per view (batch_size_per_view = 2, model.py:687): intrinsics, depth on
             views 0/2, poses on views 0/1, per-scene metric flags
  cfg1_224 under the reference's own bf16 autocast recipe, emulated on CPU (device "cuda" -> "cpu"):
             rel-L2 of bf16 vs fp32 per output key = the bf16 yardstick (golden_bf16_yardstick.json)
Info-sharing variants (the reference built with a modified info_sharing_config):
  gat_224      3 views 224x224, MultiViewGlobalAttentionTransformerIFR (24 global blocks, view PE on every view,
               sequential indices, entropy scaling) — configs/model/info_sharing/gat_ifr_24_layers_escaling.yaml
               with use_rand_idx_pe_for_non_reference_views False (the random draw is not reproducible across
               implementations' RNG use)
  aatpe_224    3 views 224x224, AAT with PE on the non-reference views too (sequential) and scalable softmax
  aatnoref_224 2 views 224x224, AAT without any view PE (distinguish_ref_and_non_ref_views False)
  aat48_224    2 views 224x224, configs/model/info_sharing/aat_ifr_48_layers_escaling.yaml: 48 blocks of width 1024
               / 16 heads (proj_embed = identity), three taps [11, 23, 35] feeding the DPT without the encoder
               features (model.py:323-330, 1748-1768), entropy scaling
"""

import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


PKG = os.path.join(REPO, "map-anything_amd", "mapanything")
synthetic = _load(os.path.join(PKG, "utils", "synthetic.py"), "mapa_synthetic")
mspec = _load(os.path.join(PKG, "models", "mapanything", "spec.py"), "mapa_spec")

OUT_KEYS = ["pts3d", "pts3d_cam", "ray_directions", "depth_along_ray", "depth_z", "cam_trans", "cam_quats",
            "metric_scaling_factor", "conf", "non_ambiguous_mask_logits", "non_ambiguous_mask", "intrinsics",
            "camera_poses", "img_no_norm"]


def synthetic_reference_state_dict(info_sharing_config=None):
    info = mspec.InfoSharingSpec.from_config(info_sharing_config)
    canon = synthetic.synthetic_state_dict(mspec.canonical_spec(info))
    sd = {k: torch.from_numpy(v) for k, v in canon.items()}
    for a, c in mspec.aliases(info).items():
        sd[a] = sd[c]
    return sd


def _info_cfg(model_type, **module_args):
    args = dict(name=f"{model_type}_variant", input_embed_dim=1024, indices=[11, 17], norm_intermediate=True,
                size="24_layers", depth=24, gradient_checkpointing=False, custom_positional_encoding=None)
    args.update(module_args)
    return {"model_type": model_type, "model_return_type": "intermediate_features",
            "custom_positional_encoding": None, "module_args": args}


VARIANTS = {
    "gat_224": (_info_cfg("global_attention", max_num_views=1000, use_rand_idx_pe_for_non_reference_views=False,
                          use_entropy_scaling=True),
                dict(views=3, h=224, w=224, seed=8)),
    "aatpe_224": (_info_cfg("alternating_attention", distinguish_ref_and_non_ref_views=True,
                            use_pe_for_non_reference_views=True, max_num_views_for_pe=1000,
                            use_rand_idx_pe_for_non_reference_views=False, use_scalable_softmax=True),
                  dict(views=3, h=224, w=224, seed=9)),
    "aatnoref_224": (_info_cfg("alternating_attention", distinguish_ref_and_non_ref_views=False),
                     dict(views=2, h=224, w=224, seed=10)),
    "aat48_224": (_info_cfg("alternating_attention", name="aat_48_layers_ifr", indices=[11, 23, 35], size="48_layers",
                            depth=48, dim=1024, num_heads=16, distinguish_ref_and_non_ref_views=True,
                            use_entropy_scaling=True),
                  dict(views=2, h=224, w=224, seed=11)),
}


def make_views(case):
    n, h, w, seed = case["views"], case["h"], case["w"], case["seed"]
    B = case.get("batch", 1)  # scenes per view (batch_size_per_view, reference model.py:687)
    imgs = synthetic.synthetic_images(n, h, w, seed, batch=B)
    views = []
    for v in range(n):
        view = {"img": torch.from_numpy(imgs[v]), "data_norm_type": ["dinov2"]}
        if case.get("multimodal"):
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed, batch=B)[v])
            view["depth_z"] = torch.from_numpy(synthetic.synthetic_sparse_depth(n, h, w, seed, batch=B)[v])
            view["is_metric_scale"] = torch.ones(B, dtype=torch.bool)
        if case.get("rays_only"):
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed, batch=B)[v])
        if case.get("mixed"):
            # 3 views: intrinsics everywhere, depth on views 0 and 2, poses on views 0 and 1; scene 0: view 2 not
            # metric, further scenes: only view 0 metric
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed, batch=B)[v])
            if v in (0, 2):
                view["depth_z"] = torch.from_numpy(synthetic.synthetic_sparse_depth(n, h, w, seed, batch=B)[v])
            if v in (0, 1):
                view["camera_poses"] = torch.from_numpy(synthetic.synthetic_poses(n, seed, batch=B)[v])
            view["is_metric_scale"] = torch.tensor([(v != 2) if b == 0 else (v == 0) for b in range(B)])
        views.append(view)
    return views


class Taps:
    def __init__(self, model):
        self.d = {}
        self.h = []
        self.h.append(model.encoder.register_forward_hook(self._enc))
        self.h.append(model.fusion_norm_layer.register_forward_hook(self._fused))
        self.h.append(model.info_sharing.register_forward_hook(self._aat))
        self.h.append(model.dpt_feature_head.register_forward_hook(self._dpt))
        self.h.append(model.dpt_regressor_head.register_forward_hook(self._reg))
        self.h.append(model.pose_head.register_forward_hook(self._pose))
        self.h.append(model.scale_head.register_forward_hook(self._scale))

    def _enc(self, m, i, o):
        self.d["tap_encoder"] = o.features.float().numpy().copy()

    def _fused(self, m, i, o):
        self.d["tap_fused_nhwc"] = o.float().numpy().copy()

    def _aat(self, m, i, o):
        final, inter = o
        self.d["tap_aat_final"] = torch.stack(final.features, 1).float().numpy().copy()
        for d, t in zip(m.indices, inter):  # the taps are named by their block index
            self.d[f"tap_aat_l{d}"] = torch.stack(t.features, 1).float().numpy().copy()
        self.d["tap_scale_token"] = final.additional_token_features.float().numpy().copy()

    def _dpt(self, m, i, o):
        self.d["tap_dpt_feature"] = o.features_upsampled_8x.float().numpy().copy()

    def _reg(self, m, i, o):
        self.d["tap_dense_raw"] = o.decoded_channels.float().numpy().copy()

    def _pose(self, m, i, o):
        self.d["tap_pose_raw"] = o.decoded_channels.float().numpy().copy()

    def _scale(self, m, i, o):
        self.d["tap_scale_raw"] = o.decoded_channels.float().numpy().copy()

    def remove(self):
        for h in self.h:
            h.remove()


def run_case(model, case, bf16=False):
    views = make_views(case)
    taps = Taps(model)
    t0 = time.time()
    if bf16:
        with cpu_autocast_emulation():
            preds = model.infer(views, apply_mask=False, use_amp=True, amp_dtype="bf16")
    else:
        preds = model.infer(views, apply_mask=False, use_amp=False)
    dt = time.time() - t0
    taps.remove()
    out = {}
    for k in OUT_KEYS:
        if k in preds[0]:
            arr = torch.stack([p[k].float() for p in preds], 0).numpy()
            out[f"out_{k}"] = arr
    out.update(taps.d)
    return out, dt


class cpu_autocast_emulation:
    """map autocast("cuda") to CPU autocast so the reference's own enabled=False
    regions (model.py:1377, 1774) stay fp32 while the rest runs bf16."""

    def __enter__(self):
        self._orig = torch.autocast
        self._bf16 = torch.cuda.is_bf16_supported
        orig = self._orig

        class _AC(orig):
            def __init__(self, device_type, *a, **k):
                super().__init__("cpu" if device_type == "cuda" else device_type, *a, **k)

        torch.autocast = _AC
        torch.cuda.is_bf16_supported = lambda *a, **k: True
        return self

    def __exit__(self, *exc):
        torch.autocast = self._orig
        torch.cuda.is_bf16_supported = self._bf16


KEEP_OUT = ("out_pts3d", "out_ray_directions", "out_depth_along_ray", "out_conf", "out_non_ambiguous_mask_logits",
            "out_cam_trans", "out_cam_quats", "out_metric_scaling_factor", "out_intrinsics", "out_camera_poses")
DENSE = ("out_pts3d", "out_ray_directions", "out_depth_along_ray", "out_conf", "out_non_ambiguous_mask_logits")
SPATIAL_TAPS_NCHW = ("tap_encoder", "tap_dpt_feature")


def shrink(d, out_step, tap_step, dpt_step):
    """Keep fixtures small: dense outputs strided by out_step, feature taps by tap_step (dpt feature by
    dpt_step). Keys derivable from kept ones (pts3d_cam, depth_z, masks, img_no_norm, raw dense) are dropped."""
    out = {}
    for k in KEEP_OUT:
        v = d[k]
        out[k] = v[:, :, ::out_step, ::out_step] if k in DENSE else v
    out["tap_encoder"] = d["tap_encoder"][:, :, ::tap_step, ::tap_step]
    out["tap_fused_nhwc"] = d["tap_fused_nhwc"][:, ::tap_step, ::tap_step, :]
    for k in d:
        if k.startswith("tap_aat_"):
            out[k] = d[k][:, :, :, ::tap_step, ::tap_step]
    out["tap_dpt_feature"] = d["tap_dpt_feature"][:, :, ::dpt_step, ::dpt_step]
    for k in ("tap_scale_token", "tap_pose_raw", "tap_scale_raw"):
        out[k] = d[k]
    return {k: np.ascontiguousarray(v) for k, v in out.items()}


STEPS = {"cfg1_224": (1, 2, 8), "v2_518": (7, 6, 24), "cfg2_518": (7, 6, 24), "cfg4_518": (14, 12, 48), "mm_224": (2, 4, 8), "mixed_224": (2, 4, 8),
         "ns_280x392": (4, 2, 8), "one_224": (2, 2, 8), "b2_224": (2, 4, 8), "gat_224": (4, 2, 8), "aatpe_224": (4, 2, 8),
         "aatnoref_224": (4, 2, 8), "aat48_224": (4, 2, 8)}


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def main():
    torch.set_num_threads(os.cpu_count())
    model = ref_harness.build_reference_model()
    sd_spec = [[k, list(v.shape)] for k, v in model.state_dict().items()]
    with open(os.path.join(HERE, "ref_state_dict_spec.json"), "w") as f:
        json.dump(sd_spec, f)
    t0 = time.time()
    sd = synthetic_reference_state_dict()
    missing, unexpected = model.load_state_dict(sd, strict=True), None
    print("synthetic weights", time.time() - t0, "s")

    meta = {}
    cases = {
        "cfg1_224": dict(views=2, h=224, w=224, seed=1),
        "v2_518": dict(views=2, h=518, w=518, seed=2),
        "mm_224": dict(views=2, h=224, w=224, seed=4, multimodal=True),
        "mixed_224": dict(views=3, h=224, w=224, seed=5, mixed=True),
        "ns_280x392": dict(views=2, h=280, w=392, seed=6),
        "one_224": dict(views=1, h=224, w=224, seed=7, rays_only=True),
        "cfg2_518": dict(views=8, h=518, w=518, seed=2),
        "cfg4_518": dict(views=32, h=518, w=518, seed=4, multimodal=True),
        "b2_224": dict(views=3, h=224, w=224, seed=12, mixed=True, batch=2),
    }
    no_bf16 = ("cfg4_518",)
    only = os.environ.get("GOLDEN_ONLY")
    variants = dict(VARIANTS)
    if only:
        cases = {k: v for k, v in cases.items() if k in only.split(",")}
        variants = {k: v for k, v in variants.items() if k in only.split(",")}
        meta = json.load(open(os.path.join(HERE, "golden_meta.json")))
    models = {name: model for name in cases}
    for name, (info_cfg, case) in variants.items():
        cfg = ref_harness.reference_config()
        cfg["info_sharing_config"] = json.loads(json.dumps(info_cfg))
        vm = ref_harness.load_reference()(**cfg).eval()
        vm.load_state_dict(synthetic_reference_state_dict(info_cfg), strict=True)
        models[name] = vm
        cases[name] = dict(case, info_sharing_config=info_cfg)
    fp32 = {}
    for name, case in cases.items():
        model = models[name]
        out, dt = run_case(model, case)
        fp32[name] = out
        meta[name] = dict(case, seconds=dt)
        out = shrink(out, *STEPS[name])
        meta[name]["steps_out_tap_dpt"] = STEPS[name]
        np.savez_compressed(os.path.join(HERE, f"golden_{name}.npz"), **out)
        print(name, f"{dt:.2f}s", {k: v.shape for k, v in out.items()})

    # bf16 yardsticks (reference's own bf16 recipe vs its fp32 path), per case
    ypath = os.path.join(HERE, "golden_bf16_yardsticks.json")
    yards = json.load(open(ypath)) if os.path.exists(ypath) else {}
    for name in cases:
        if name in no_bf16:
            continue
        try:
            out16, dt16 = run_case(models[name], cases[name], bf16=True)
        except RuntimeError as e:
            # aatnoref_224: without any view PE the proj_embed output stays bf16 into the autocast-disabled heads
            # (model.py:1774) and the reference's own bf16 path fails there ("Input type (c10::BFloat16) and bias
            # type (float) should be the same", dpt.py:210); the GPU test then uses cfg1's yardstick
            yards[name] = {"reference_bf16_error": str(e).splitlines()[0]}
            continue
        yard = {"seconds": dt16}
        for k, v in out16.items():
            if v.dtype == np.bool_:
                yard[k] = float(np.mean(v != fp32[name][k]))
            else:
                yard[k] = rel_l2(v, fp32[name][k])
        yards[name] = yard
    with open(ypath, "w") as f:
        json.dump(yards, f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("done")


if __name__ == "__main__":
    main()

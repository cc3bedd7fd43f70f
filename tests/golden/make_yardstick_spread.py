"""Spread of the reference's own bf16-vs-fp32 deviation, per case (run in the build container only).

    python tests/golden/make_yardstick_spread.py            # writes tests/golden/golden_bf16_spread.json
    GOLDEN_ONLY=cfg4_518 python tests/golden/make_yardstick_spread.py
    SPREAD_AMP=fp16 GOLDEN_ONLY=cfg1_224,mm_224,v2_518,cfg2_518 python tests/golden/make_yardstick_spread.py
                                                            # the fp16 autocast recipe -> golden_fp16_spread.json

One bf16 run of the reference is ONE sample of its bf16 rounding walk: a scalar output such as
metric_scaling_factor (one number per scene) can land anywhere inside a spread several times wide.  To measure that
spread, the reference's own `infer` (bf16 autocast recipe, emulated on CPU exactly as make_golden.py does) is run on
the case's inputs with the images perturbed by relative noise of 2^-20 (far below anything the fp32 path resolves:
the fp32 output moves by `perturbation_fp32_effect`, recorded for cfg1) under SAMPLES seeds plus the unperturbed
input, and each run's rel-L2 against the committed fp32 fixture (same subsampling as the GPU test) is stored.
tests/test_gpu_model.py bounds every output of every case by its OWN case's spread (max over the samples).

The info-sharing variants (make_golden.py VARIANTS) are covered the same way, except aatnoref_224, whose bf16
path fails inside the reference itself.  cfg4_518 (32 views 518^2 multimodal) also gets its own unperturbed yardstick in golden_bf16_yardsticks.json (the
CPU bf16 emulation takes ~2.5 min per run here; round 2 borrowed cfg2's).
"""

import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402
import ref_harness  # noqa: E402

SAMPLES = int(os.environ.get("SPREAD_SAMPLES", "5"))
AMP = os.environ.get("SPREAD_AMP", "bf16")  # the autocast dtype of the recipe whose spread is measured: bf16 / fp16
REL_NOISE = 2.0 ** -20
SMALL = ("out_cam_trans", "out_cam_quats", "out_metric_scaling_factor", "out_camera_poses", "out_intrinsics")

CASES = {
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


def perturbed_views(case, pseed):
    views = mg.make_views(case)
    if pseed is None:
        return views
    g = torch.Generator().manual_seed(1000 + pseed)
    for v in views:
        img = v["img"]
        v["img"] = img * (1.0 + REL_NOISE * torch.randn(img.shape, generator=g, dtype=img.dtype))
    return views


def run(model, case, pseed, bf16=True):
    views = perturbed_views(case, pseed)
    if bf16:
        with mg.cpu_autocast_emulation():
            preds = model.infer(views, apply_mask=False, use_amp=True, amp_dtype=AMP)
    else:
        preds = model.infer(views, apply_mask=False, use_amp=False)
    out = {}
    for k in mg.KEEP_OUT:
        key = k[len("out_"):]
        arr = torch.stack([p[key].float() for p in preds], 0).numpy()
        out[k] = arr
    return out


# outputs multiplied by the scene's metric_scaling_factor (model.py:1911-1921): compared also with each side's own
# factor divided out ("_unscaled"), so their scale-free part can be held to the dense tolerance and the scalar's
# one-number noise is accounted for once, in metric_scaling_factor itself
METRIC = ("out_pts3d", "out_depth_along_ray", "out_cam_trans", "out_camera_poses")


def unscale(k, v, s):
    """v / s per (view, scene): s = metric_scaling_factor (V, B, 1); camera_poses: translation column only."""
    s = np.asarray(s, np.float64).reshape(s.shape[0], s.shape[1])
    v = np.asarray(v, np.float64).copy()
    if k == "out_camera_poses":
        v[..., :3, 3] /= s[:, :, None]
        return v
    return v / s.reshape(s.shape + (1,) * (v.ndim - 2))


def compare(out, fix, step):
    res = {}
    for k in mg.KEEP_OUT:
        v = out[k]
        if k in mg.DENSE:
            v = v[:, :, ::step, ::step]
        res[k] = mg.rel_l2(v, fix[k])
        if k in METRIC:
            res[k + "_unscaled"] = mg.rel_l2(unscale(k, v, out["out_metric_scaling_factor"]),
                                             unscale(k, fix[k], fix["out_metric_scaling_factor"]))
    return res


def main():
    torch.set_num_threads(os.cpu_count())
    only = os.environ.get("GOLDEN_ONLY")
    cases = {k: v for k, v in CASES.items() if not only or k in only.split(",")}
    variants = {k: v for k, v in mg.VARIANTS.items() if not only or k in only.split(",")}
    model = ref_harness.build_reference_model()
    model.load_state_dict(mg.synthetic_reference_state_dict(), strict=True)
    models = {name: model for name in cases}
    for name, (info_cfg, case) in variants.items():
        if name == "aatnoref_224":  # the reference's own bf16 path fails on this variant (make_golden.py)
            continue
        cfg = ref_harness.reference_config()
        cfg["info_sharing_config"] = json.loads(json.dumps(info_cfg))
        vm = ref_harness.load_reference()(**cfg).eval()
        vm.load_state_dict(mg.synthetic_reference_state_dict(info_cfg), strict=True)
        models[name] = vm
        cases[name] = case
    spath = os.path.join(HERE, f"golden_{AMP}_spread.json")
    spread = json.load(open(spath)) if os.path.exists(spath) else {}
    ypath = os.path.join(HERE, "golden_bf16_yardsticks.json")
    yards = json.load(open(ypath))
    for name, case in cases.items():
        fix = np.load(os.path.join(HERE, f"golden_{name}.npz"))
        step = mg.STEPS[name][0]
        t0 = time.time()
        samples = {}
        for pseed in [None] + list(range(SAMPLES)):
            r = compare(run(models[name], case, pseed), fix, step)
            for k, e in r.items():
                samples.setdefault(k, []).append(e)
            if pseed is None and name not in yards and AMP == "bf16":
                yards[name] = dict(r, seconds=time.time() - t0, note="unperturbed reference bf16 run vs the fp32 fixture "
                                   "(make_yardstick_spread.py; fixture subsampling)")
        entry = {"samples": 1 + SAMPLES, "rel_noise": REL_NOISE, "seconds": time.time() - t0,
                 "rel_l2": samples, "max": {k: max(v) for k, v in samples.items()},
                 "min": {k: min(v) for k, v in samples.items()}}
        if name == "cfg1_224":
            # how far the perturbation alone moves the fp32 path (must be << every bf16 sample)
            entry["perturbation_fp32_effect"] = compare(run(models[name], case, 0, bf16=False), fix, step)
        spread[name] = entry
        print(name, f"{entry['seconds']:.1f}s", {k[4:]: f"{min(v):.2e}..{max(v):.2e}" for k, v in samples.items()},
              flush=True)
        with open(spath, "w") as f:
            json.dump(spread, f, indent=1, sort_keys=True)
        if AMP == "bf16":
            with open(ypath, "w") as f:
                json.dump(yards, f, indent=1, sort_keys=True)
    print("done")


if __name__ == "__main__":
    main()

"""Our engine's own bf16-vs-fp32-fixture deviation on the perturbed inputs of make_yardstick_spread.py (same noise
draw), next to the reference's recorded spread: python tools/spread_gpu.py aatpe_224 gat_224 ..."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "map-anything_amd"), os.path.join(REPO, "tests")]
from tests_helpers import CASES, VARIANT_CASES, make_views, released_config, variant_config  # noqa: E402

KEYS = ("pts3d", "ray_directions", "depth_along_ray", "conf", "cam_trans", "cam_quats", "metric_scaling_factor")


def perturbed(case, pseed):
    views = make_views(case)
    if pseed is None:
        return views
    g = torch.Generator().manual_seed(1000 + pseed)
    for v in views:
        img = v["img"]
        v["img"] = img * (1.0 + 2.0 ** -20 * torch.randn(img.shape, generator=g, dtype=img.dtype))
    return views


def main():
    from mapanything.models import MapAnything

    spread = json.load(open(os.path.join(REPO, "tests", "golden", "golden_bf16_spread.json")))
    meta = json.load(open(os.path.join(REPO, "tests", "golden", "golden_meta.json")))
    for name in sys.argv[1:]:
        if name in VARIANT_CASES:
            cfg, case = variant_config(name)
        else:
            cfg, case = released_config(), CASES[name]
        m = MapAnything(**cfg).load_synthetic_weights().to("cuda").eval()
        g = np.load(os.path.join(REPO, "tests", "golden", f"golden_{name}.npz"))
        step = meta[name]["steps_out_tap_dpt"][0]
        ours = {k: [] for k in KEYS}
        for pseed in [None] + list(range(5)):
            preds = m.infer(perturbed(case, pseed), apply_mask=False)
            for k in KEYS:
                mine = torch.stack([p[k].float() for p in preds], 0).cpu().numpy().astype(np.float64)
                if mine.ndim >= 4:
                    mine = mine[:, :, ::step, ::step]
                ref = g[f"out_{k}"].astype(np.float64)
                ours[k].append(float(np.linalg.norm(mine - ref) / np.linalg.norm(ref)))
        print(f"[{name}] ours median / max  vs  reference median / max (6 samples each)")
        for k in KEYS:
            r = spread[name]["rel_l2"][f"out_{k}"]
            print(f"  {k:24s} {np.median(ours[k]):.3e} / {max(ours[k]):.3e}   {np.median(r):.3e} / {max(r):.3e}"
                  f"   median ratio {np.median(ours[k]) / np.median(r):.2f}", flush=True)


if __name__ == "__main__":
    main()

"""Locate non-finite values in the engine's outputs (debug aid): python tools/nan_probe.py <case> <precision>"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "map-anything_amd"), os.path.join(REPO, "tests")]
from tests_helpers import CASES, make_views, released_config  # noqa: E402


def main():
    from mapanything.models import MapAnything

    name, prec = sys.argv[1], sys.argv[2]
    m = MapAnything(**released_config()).load_synthetic_weights().to("cuda").eval()
    eng = m.engine(prec)
    views = make_views(CASES[name])
    imgs = torch.cat([v["img"] for v in views], 0).cuda()
    taps = {}
    out = eng.run(imgs, taps=taps)
    for k, v in list(out.items()) + [("tap_" + k, v) for k, v in taps.items() if torch.is_tensor(v)]:
        if not torch.is_tensor(v) or not v.is_floating_point():
            continue
        bad = ~torch.isfinite(v)
        n = int(bad.sum())
        print(f"{k:28s} {tuple(v.shape)} nonfinite {n}" + (f" first at {bad.nonzero()[:3].tolist()}" if n else "")
              + f"  max|v| {float(v[torch.isfinite(v)].abs().max()):.3e}", flush=True)
    rays = out["ray_directions"]
    z0 = (rays[..., 2] == 0).nonzero().tolist()
    print("rays z == 0:", len(z0), z0[:8], " min |z|:", float(rays[..., 2].abs().min()))
    for v, y, x in z0[:4]:
        print("  ray", rays[v, y, x].tolist(), "depth", float(out["depth_along_ray"][v, y, x, 0]),
              "pts3d_cam", out["pts3d_cam"][v, y, x].tolist())


if __name__ == "__main__":
    main()

"""Debug aid: the regressor's raw 6-channel output at pixels whose ray z came out exactly 0 (fp16 v2_518)."""
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
    imgs = torch.cat([v["img"] for v in make_views(CASES[name])], 0).cuda()
    fused = eng.run(imgs)
    os.environ["MAPA_FUSED_HEAD"] = "0"
    unf = eng.run(imgs)
    for tag, o in (("fused", fused), ("unfused", unf)):
        z0 = (o["ray_directions"][..., 2] == 0).nonzero().tolist()
        print(tag, "z==0 at", z0, "min|z|", float(o["ray_directions"][..., 2].abs().min()))
    d = (fused["ray_directions"] - unf["ray_directions"]).abs().max()
    print("max |fused - unfused| rays", float(d))
    # raw = hidden @ w6^T + b6 from the unfused hidden map (fp32 in split mode)
    V, H, W = imgs.shape[0], imgs.shape[2], imgs.shape[3]
    from mapanything import _native as nat  # noqa: F401
    hp, wp = H // 14, W // 14
    T = hp * wp
    fl, ff, tok = None, None, None
    for v, y, x in (fused["ray_directions"][..., 2] == 0).nonzero().tolist():
        print(" fused ray", fused["ray_directions"][v, y, x].tolist(), " unfused ray", unf["ray_directions"][v, y, x].tolist())


if __name__ == "__main__":
    main()

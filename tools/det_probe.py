"""Determinism probe: the bf16 engine run twice (and a third time) on identical inputs must agree bit for bit at
every stage tap and output; prints the first stage that differs.  Also repeats single kernels (attention at the 2-view
224^2 global shape, the fused regressor-head conv) on fixed inputs.  python tools/det_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from mapanything.models import MapAnything  # noqa: E402
from tests_helpers import released_config, make_views  # noqa: E402


def cmp(a, b, label):
    bad = []
    for k in a:
        x, y = a[k], b[k]
        if isinstance(x, torch.Tensor) and not torch.equal(x, y):
            d = (x.float() - y.float()).abs()
            bad.append((k, int((d > 0).sum()), float(d.max())))
            if x.dim() >= 3:
                idx = (d.reshape(d.shape[0], d.shape[1], d.shape[2], -1).amax(-1) > 0).nonzero()[:40].tolist()
                print("   ", k, "differing (view, y, x):", idx, flush=True)
                i0 = tuple(idx[0])
                print("   ", k, "values", x[i0].tolist(), y[i0].tolist(), flush=True)
    print(label, "identical" if not bad else bad[:12], flush=True)
    return bad


def main():
    torch.manual_seed(0)
    model = MapAnything(**released_config(), precision="bf16").load_synthetic_weights().cuda().eval()
    for (nv, hw) in ((8, 518), (8, 518)):
        views = make_views(dict(views=nv, h=hw, w=hw, seed=11))
        imgs = torch.cat([v["img"] for v in views], 0).cuda()
        eng = model.engine("bf16")
        runs = []
        for r in range(3):
            taps = {}
            out = eng.run(imgs, taps=taps)
            torch.cuda.synchronize()
            runs.append(({k: v.clone() for k, v in taps.items() if isinstance(v, torch.Tensor)},
                         {k: v.clone() for k, v in out.items()}))
        for r in (1, 2):
            cmp(runs[0][0], runs[r][0], f"{nv}x{hw} taps run0 vs run{r}:")
            cmp(runs[0][1], runs[r][1], f"{nv}x{hw} outputs run0 vs run{r}:")


if __name__ == "__main__":
    main()

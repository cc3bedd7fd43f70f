"""Same-process A/B of whole-model infer() on one GPU (the guide's rule: interleaved rounds, medians), for packing-time
switches.  Usage: python tools/ab_model.py kblock [views] [rounds] [steps]
  kblock: head convs with the channel-block-major K order (engine.KBLOCK = 32) vs tap-major (0);
  halo: stride-1 head convs on the LDS halo-window kernel vs the implicit GEMM;
  tailsk: tail-only stream-K for the GEMMs with a nearly empty last wave vs data-parallel;
  fusedhead: the regressor's conv2 carrying the dense head (mapa_regressor_head_out) vs conv + dense_head_out."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "map-anything_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from mapanything.models import MapAnything  # noqa: E402
from mapanything.models.mapanything import engine  # noqa: E402
from mapanything.utils import synthetic  # noqa: E402
from tests_helpers import released_config  # noqa: E402


def main():
    what = sys.argv[1]
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    dev = torch.device("cuda", 0)
    imgs = synthetic.synthetic_images(V, 518, 518, seed=2)
    views = [{"img": torch.from_numpy(i).to(dev), "data_norm_type": ["dinov2"]} for i in imgs]
    from mapanything import _native as nat

    if what == "kblock":
        arms = [("kblock32", lambda: setattr(engine, "KBLOCK", 32)), ("tapmajor", lambda: setattr(engine, "KBLOCK", 0))]
    elif what == "halo":  # the kernel choice is baked into each model's captured graph at its first infer
        arms = [("halo", lambda: nat.gemm_tune(nat.TUNE_CONV_HALO, 1)),
                ("implicit", lambda: nat.gemm_tune(nat.TUNE_CONV_HALO, 0))]
    elif what == "halo8":  # N = 256 halo convs: 8x16-pixel blocks / 256-wide tiles vs 16x16 / 128-wide
        arms = [("rows8", lambda: nat.gemm_tune(nat.TUNE_CONV_HALO, 1)),
                ("rows16", lambda: nat.gemm_tune(nat.TUNE_CONV_HALO, 2))]
    elif what == "flat":  # 19^2 / 37^2 stride-1 head convs: flat-raster split-K halo conv vs stream-K implicit GEMM
        arms = [("flat", lambda: nat.gemm_tune(nat.TUNE_CONV_HALO, 1)),
                ("streamk", lambda: nat.gemm_tune(nat.TUNE_CONV_HALO, 3))]
    elif what == "tailsk":
        arms = [("tailsk", lambda: nat.gemm_tune(nat.TUNE_TAIL_STREAMK, 1)),
                ("dataparallel", lambda: nat.gemm_tune(nat.TUNE_TAIL_STREAMK, 0))]
    elif what == "fusedhead":
        arms = [("fused", lambda: os.environ.__setitem__("MAPA_FUSED_HEAD", "1")),
                ("twolaunch", lambda: os.environ.__setitem__("MAPA_FUSED_HEAD", "0"))]
    elif what == "headbranch":  # pose / scale heads on a side-stream branch vs in line
        arms = [("branch", lambda: os.environ.__setitem__("MAPA_HEAD_BRANCH", "1")),
                ("inline", lambda: os.environ.__setitem__("MAPA_HEAD_BRANCH", "0"))]
    elif what == "heads":  # TF32-equivalent heads (f16 x2) vs fp32-exact split bf16 heads (x3) vs bf16 fast mode
        arms = [(h, (lambda h=h: os.environ.__setitem__("MAPA_AB_HEADS", h))) for h in ("tf32", "tf32x2", "fp32", "bf16")]
    elif what == "lnfuse":  # residual linears with the next LayerNorm fused: all / N % 256 only / none
        arms = [("all", lambda: nat.gemm_tune(nat.TUNE_LN_FUSE, 2)), ("n256", lambda: nat.gemm_tune(nat.TUNE_LN_FUSE, 3)),
                ("none", lambda: nat.gemm_tune(nat.TUNE_LN_FUSE, 0))]
    else:
        raise SystemExit(f"unknown A/B {what}")
    models, sd = [], None
    for name, setup in arms:
        setup()
        m = MapAnything(**released_config(), head_precision=os.environ.get("MAPA_AB_HEADS", "tf32")).to(dev).eval()
        if sd is None:
            m.load_synthetic_weights()
            sd = m._sd
        else:
            m._sd = sd
        for _ in range(2):
            m.infer(views)  # packs the weights under this arm's switch, captures the graph
        models.append((name, m, setup))
    torch.cuda.synchronize()
    ts = {n: [] for n, _, _ in models}
    for _ in range(rounds):
        for n, m, setup in models:
            setup()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                m.infer(views)
            torch.cuda.synchronize()
            ts[n].append((time.perf_counter() - t0) / steps * 1e3)
    for n, t in ts.items():
        t = sorted(t)
        print(f"{what} {n:10s} median {t[len(t) // 2]:7.2f} ms/infer  min {t[0]:7.2f}  ({V * 1e3 / t[len(t) // 2]:.1f} views/s)")


if __name__ == "__main__":
    main()

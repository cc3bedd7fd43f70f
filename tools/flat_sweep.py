"""Flat-raster split-K halo conv (variant 2589) against the stream-K implicit GEMM (2580/2581) on the DPT's small-map
head convs at 8 views, with a sweep of the K part count (mapa_gemm_tune(MAPA_TUNE_HALO_SPLIT)).  Interleaved in one
process (tools/kbench.py's rule).  FS_F16=1: the TF32-equivalent heads' plain binary16 operands (logical channel
widths).  Usage: python tools/flat_sweep.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

V = 8
# name, H, W, C (per-pixel operand width: 3x the logical channels of the split-precision convs), Co
CONVS = [("l3rn@37", 37, 37, 1152, 256), ("l4rn@19", 19, 19, 2304, 256), ("rn4@19", 19, 19, 768, 256),
         ("rn3@37", 37, 37, 768, 256)]
DT = torch.bfloat16
if os.environ.get("FS_F16"):
    CONVS = [("l3rn@37", 37, 37, 384, 256), ("l4rn@19", 19, 19, 768, 256), ("rn4@19", 19, 19, 256, 256),
             ("rn3@37", 37, 37, 256, 256)]
    DT = torch.float16
SPLITS = [int(s) for s in os.environ.get("FS_SPLITS", "0,2,3,4,6,8").split(",")]
ROUNDS = 3


def timeit(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    nat.lib()
    for name, H, W, C, Co in CONVS:
        x = (torch.randn(V, H, W, C, device="cuda") * 0.5).to(DT)
        w = (torch.randn(Co, 9 * C, device="cuda") * (9 * C) ** -0.5).to(DT)
        w = w.view(Co, 9, C // 32, 32).permute(0, 2, 1, 3).contiguous().reshape(Co, -1)
        w._mapa_kblock = 32
        b = torch.randn(Co, device="cuda")
        o = torch.empty(V * H * W, Co, device="cuda", dtype=DT)
        M = V * H * W
        sk = 2581 if Co >= 512 and M >= 2048 else 2580

        def run(var, split):
            def f():
                nat.gemm_set_variant(var)
                nat.gemm_tune(nat.TUNE_HALO_SPLIT, split)
                nat.gemm(x, w, M, Co, 9 * C, bias=b, out_lp=o, conv=(C, H, W, H, W, 1))
            return f
        combos = [(sk, 0)] + [(2589, s) for s in SPLITS]
        ts = [[] for _ in combos]
        for _ in range(ROUNDS):
            for i, (v, s) in enumerate(combos):
                ts[i].append(timeit(run(v, s), reps))
        for (v, s), t in zip(combos, ts):
            ms = sorted(t)[len(t) // 2]
            print(f"{name:9s} v{v} split {s:2d}: {ms*1e3:8.1f} us  {2*M*Co*9*C/ms/1e9:7.1f} TF/s", flush=True)
        nat.gemm_set_variant(0)
        nat.gemm_tune(nat.TUNE_HALO_SPLIT, 0)


if __name__ == "__main__":
    main()

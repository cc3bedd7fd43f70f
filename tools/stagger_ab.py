"""A/B of the persistent GEMM's start stagger (mapa_gemm_tune MAPA_TUNE_PERS_STAGGER: the workgroups with one tile
fewer start late, so the chip's epilogue store bursts stop coinciding) and of its tile shapes (SA_SHAPES: forced
variants 2600 + shape) on the path's transformer linears (8 views, 518^2), interleaved in one process; every output
is checked bitwise against the first configuration's.
Usage: python tools/stagger_ab.py [reps] [out.json] [ticks,ticks,...]   (SA_SHAPES=3,7,8: shapes x ticks)"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

if os.environ.get("MAPA_AB_LIB"):  # A/B builds (tools/ab_build.sh): load before any other call
    nat.load_library(os.environ["MAPA_AB_LIB"])

V, T = 8, 1369
R, L = V * (T + 1), V * T + 1
SHAPES = [("enc.qkv", R, 3072, 1024, "plain"), ("enc.fc1", R, 4096, 1024, "gelu"), ("aat.qkv", L, 2304, 768, "plain"),
          ("aat.fc1", L, 3072, 768, "gelu"), ("enc.fc2", R, 1024, 4096, "resid"), ("aat.fc2", L, 768, 3072, "resid"),
          ("enc.proj", R, 1024, 1024, "resid"), ("aat.proj", L, 768, 768, "resid")]
if os.environ.get("SA_ONLY"):
    SHAPES = [s for s in SHAPES if s[0] in os.environ["SA_ONLY"].split(",")]


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
    return s.elapsed_time(e) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    out_path = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/stagger_ab.json"
    ticks = [int(t) for t in (sys.argv[3] if len(sys.argv) > 3 else "0,500,1000,1500,2000,3000").split(",")]
    shapes = [int(x) for x in os.environ.get("SA_SHAPES", "-1").split(",")]
    confs = [(sh, t) for sh in shapes for t in ticks]
    res = {}
    for name, M, N, K, epi in SHAPES:
        A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        gam = torch.randn(N, device="cuda") * 0.1
        x0 = torch.randn(M, N, device="cuda")
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        x = x0.clone()

        def run(conf, check=False):
            sh, st = conf

            def f(check=check):
                nat.gemm_tune(nat.TUNE_PERS_STAGGER, st)
                # the residual pattern takes the persistent kernel only when forced (shape 3: 192x128, 2 / CU)
                nat.gemm_set_variant(2600 + sh if sh >= 0 else 2603 if epi == "resid" else 0)
                if epi == "resid":
                    if check:
                        x.copy_(x0)
                    nat.gemm(A, W, M, N, K, bias=b, gamma=gam, resid1=x, out_f32=x)
                    return x
                nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU if epi == "gelu" else nat.ACT_NONE, out_lp=o)
                return o
            return f

        outs = {c: run(c)(check=True).clone() for c in confs}
        fns = {c: run(c) for c in confs}
        ts = {c: [] for c in confs}
        for _ in range(3):
            for c in confs:
                ts[c].append(timeit(fns[c], reps))
        nat.gemm_tune(nat.TUNE_PERS_STAGGER, 0)
        nat.gemm_set_variant(0)
        case = {}
        for c in confs:
            us = sorted(ts[c])[1]
            same = torch.equal(outs[c], outs[confs[0]])
            case[f"s{c[0]}_t{c[1]}"] = {"us": round(us, 2), "tflops": round(2.0 * M * N * K / us / 1e6, 1),
                                        "bitwise": same}
            print(f"{name:9s} shape {c[0]:2d} stagger {c[1]:5d} ticks {us:8.1f} us {2.0*M*N*K/us/1e6:7.1f} TF/s  "
                  f"bitwise={same}", flush=True)
        res[name] = case
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()

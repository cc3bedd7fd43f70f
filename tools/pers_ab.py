"""A/B of the persistent register-epilogue GEMM (gemm_pers.hip) against the data-parallel tile kernels on the path's
transformer linears (8 views, 518^2), interleaved in one process, with a bitwise / tolerance check of the outputs.
Usage: python tools/pers_ab.py [reps] [out.json]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

V, T = 8, 1369
R, L = V * (T + 1), V * T + 1
SHAPES = [("enc.qkv", R, 3072, 1024, "plain"), ("enc.fc1", R, 4096, 1024, "gelu"), ("enc.proj", R, 1024, 1024, "resid"),
          ("enc.fc2", R, 1024, 4096, "resid"), ("aat.qkv", L, 2304, 768, "plain"), ("aat.fc1", L, 3072, 768, "gelu"),
          ("aat.proj", L, 768, 768, "resid"), ("aat.fc2", L, 768, 3072, "resid")]
if os.environ.get("PA_ONLY"):
    SHAPES = [s for s in SHAPES if s[0] in os.environ["PA_ONLY"].split(",")]


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
    out_path = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pers_ab.json"
    res = {}
    for name, M, N, K, epi in SHAPES:
        A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        gam = torch.randn(N, device="cuda") * 0.1
        x0 = torch.randn(M, N, device="cuda")
        outs = {}

        lnw, lnb = torch.randn(N, device="cuda"), torch.randn(N, device="cuda")

        def run(pers, var, ln=None):
            o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            x = x0.clone()
            lo = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

            def f(check=False):
                nat.gemm_tune(nat.TUNE_PERS, pers)
                nat.gemm_set_variant(var)
                if ln is not None:  # the residual linear + the next LayerNorm (0: gemm_big LNF tiles, 1: persistent)
                    nat.gemm_tune(nat.TUNE_PERS_LN, ln)
                    if check:
                        x.copy_(x0)
                    nat.gemm(A, W, M, N, K, bias=b, gamma=gam, resid1=x, out_f32=x, ln=(lnw, lnb, 1e-6, lo))
                    nat.gemm_tune(nat.TUNE_PERS_LN, 1)
                    return lo
                if epi == "resid":
                    if check:
                        x.copy_(x0)
                    nat.gemm(A, W, M, N, K, bias=b, gamma=gam, resid1=x, out_f32=x)
                else:
                    nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU if epi == "gelu" else nat.ACT_NONE, out_lp=o)
                return x if epi == "resid" else o
            return f
        shapes = [0, 3, 4, 5, 6] if epi != "resid" else [0, 3]  # 4-6: setprio / no-epilogue diagnostics (mode 1)
        combos = [("tiles", 0, 0), ("pers_auto", 1, 0)] + [(f"pers_s{s}", 0, 2600 + s) for s in shapes]
        fns = [run(p, v) for _, p, v in combos]
        if epi == "resid":  # LayerNorm-fused forms (compared with each other: "ln_big" is their reference)
            combos += [("ln_big", 0, 0), ("ln_pers", 0, 0)]
            fns += [run(1, 0, ln=0), run(1, 0, ln=1)]
        for (tag, _, _), f in zip(combos, fns):  # outputs once (the residual ones from the same start)
            outs[tag] = f(check=True).clone()
        ts = {c[0]: [] for c in combos}
        for _ in range(3):
            for (tag, _, _), f in zip(combos, fns):
                ts[tag].append(timeit(f, reps))
        nat.gemm_tune(nat.TUNE_PERS, 1)
        nat.gemm_set_variant(0)
        case = {}
        for tag, v in ts.items():
            us = sorted(v)[1]
            rt = "ln_big" if tag.startswith("ln_") else "tiles"
            d = (outs[tag].float() - outs[rt].float()).abs().max().item()
            same = torch.equal(outs[tag], outs[rt])
            case[tag] = {"us": round(us, 2), "tflops": round(2.0 * M * N * K / us / 1e6, 1), "bitwise": same,
                         "max_abs_diff": d}
            print(f"{name:9s} {tag:10s} {us:8.1f} us {2.0*M*N*K/us/1e6:7.1f} TF/s  bitwise={same} maxdiff={d:.3g}",
                  flush=True)
        res[name] = case
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()

"""Dense GEMM time breakdown per path shape (profiles/r6/gemm_breakdown.json): the automatic kernel, the same kernel
without its epilogue, compute-only (no K-tile reloads) and loads-only (no MFMA), K doubled, and the grid truncated to
whole waves of resident workgroups — so main-loop rate, epilogue cost and last-wave (quantisation) cost separate.
Usage: python tools/gemm_breakdown.py [out.json] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

V, T = 8, 1369
R, L = V * (T + 1), V * T + 1
# name, M, N, K, epilogue, automatic variant, its diagnostic variants (compute-only, loads-only, no-epilogue),
# workgroups resident per wave (CUs x occupancy)
SHAPES = [("enc.qkv", R, 3072, 1024, "plain", 2574, (2594, 2595, 2596), 256, 192, 256),
          ("enc.fc1", R, 4096, 1024, "gelu", 2570, (2591, 2592, 2593), 512, 256, 128),
          ("aat.qkv", L, 2304, 768, "plain", 2571, (2591, 2592, 2593), 512, 256, 128),
          ("aat.fc1", L, 3072, 768, "gelu", 2570, (2591, 2592, 2593), 512, 256, 128)]


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
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gemm_breakdown.json"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rounds = 3
    res = {}
    for name, M, N, K, epi, auto, diag, slots, bm, bn in SHAPES:
        case = {}
        ntiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
        full = (ntiles // slots) * slots
        for KK in (K, 2 * K):
            A = (torch.randn(M, KK, device="cuda") * 0.5).to(torch.bfloat16)
            W = (torch.randn(N, KK, device="cuda") * KK ** -0.5).to(torch.bfloat16)
            b = torch.randn(N, device="cuda")
            o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            act = nat.ACT_GELU if epi == "gelu" else nat.ACT_NONE

            def run(var, grid=0):
                def f():
                    nat.gemm_set_variant(var)
                    nat.gemm_tune(nat.TUNE_DIAG_GRID, grid)
                    nat.gemm(A, W, M, N, KK, bias=b, act=act, out_lp=o)
                return f
            combos = [("auto", auto, 0), ("no_epilogue", diag[2], 0), ("compute_only", diag[0], 0),
                      ("loads_only", diag[1], 0), ("full_waves", auto, full),
                      ("full_waves_no_epilogue", diag[2], full)]
            if KK != K:
                combos = combos[:2]
            ts = {c[0]: [] for c in combos}
            for _ in range(rounds):
                for tag, var, grid in combos:
                    ts[tag].append(timeit(run(var, grid), reps))
            nat.gemm_tune(nat.TUNE_DIAG_GRID, 0)
            nat.gemm_set_variant(0)
            for tag, v in ts.items():
                us = sorted(v)[len(v) // 2]
                frac_tiles = full / ntiles if tag.startswith("full_waves") else 1.0
                tf = 2.0 * M * N * KK * frac_tiles / us / 1e6
                case[f"K{KK}:{tag}"] = {"us": round(us, 2), "tflops": round(tf, 1)}
                print(f"{name:8s} K={KK:5d} {tag:24s} {us:8.1f} us {tf:7.1f} TF/s", flush=True)
        a, ne = case[f"K{K}:auto"]["us"], case[f"K{K}:no_epilogue"]["us"]
        a2, ne2 = case[f"K{2*K}:auto"]["us"], case[f"K{2*K}:no_epilogue"]["us"]
        fw = case[f"K{K}:full_waves"]["us"]
        case["derived"] = {
            "tiles": ntiles, "resident_slots": slots, "waves": round(ntiles / slots, 3), "full_wave_tiles": full,
            "epilogue_us": round(a - ne, 2),
            "main_loop_us_per_K": round((ne2 - ne) / K, 4),
            "main_loop_tflops": round(2.0 * M * N * K / (ne2 - ne) / 1e6, 1),
            "fixed_us": round(ne - (ne2 - ne), 2),
            "last_wave_us": round(a - fw, 2),
            "kernel": auto, "tile": f"{bm}x{bn}",
        }
        print(name, json.dumps(case["derived"]), flush=True)
        res[name] = case
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

"""Kernel micro-benchmark: TFLOP/s of the hot GEMM / conv / attention shapes of the 8-view 518x518 workload
(HIP-event timing, random data).  Usage: python tools/kbench.py [gemm|attn|conv|all] [reps]
KB_VARIANTS=0,2580,2568 sweeps GEMM/conv kernel variants (0 = the automatic choice; include/mapa.h); KB_KBLOCK=0,32 runs
the convs in the tap-major and the channel-block-major K order (interleaved); KB_GM=2,4,8 sweeps the 256-row GEMM
kernels' tile-group height (mapa_gemm_tune MAPA_TUNE_TILE_GROUP, interleaved with the variants)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

if os.environ.get("MAPA_AB_LIB"):  # A/B builds (tools/ab_build.sh): load before any other call
    nat.load_library(os.environ["MAPA_AB_LIB"])

nat.lib()
V, T = 8, 1369
R, L = V * (T + 1), V * T + 1
GEMMS = [("enc.qkv", R, 3072, 1024), ("enc.proj", R, 1024, 1024), ("enc.fc1", R, 4096, 1024),
         ("enc.fc2", R, 1024, 4096), ("aat.qkv", L, 2304, 768), ("aat.proj", L, 768, 768),
         ("aat.fc1", L, 3072, 768), ("aat.fc2", L, 768, 3072), ("pose.res", V * T, 784, 784)]
if os.environ.get("KB_SQ"):
    GEMMS = [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192)]
if os.environ.get("KB_SHAPES"):  # "M,N,K;M,N,K" ad-hoc GEMM shapes
    GEMMS = [(f"{m}x{n}x{k}", int(m), int(n), int(k))
             for m, n, k in (t.split(",") for t in os.environ["KB_SHAPES"].split(";"))]
ONLY = os.environ.get("KB_ONLY")
VARIANTS = [int(v) for v in os.environ.get("KB_VARIANTS", "0").split(",")]
GMS = [int(v) for v in os.environ.get("KB_GM", "0").split(",")]
if ONLY:
    GEMMS = [g for g in GEMMS if g[0] in ONLY.split(",")]
CONVS = [("rn1.c@148", V, 148, 148, 256, 256), ("reg.c2@518", V, 518, 518, 128, 128),
         ("reg.c1@296", V, 296, 296, 256, 128), ("rn2.c@74", V, 74, 74, 256, 256)]
if os.environ.get("KB_CONVS"):  # "name,n,H,W,C,Co;..." ad-hoc 3x3 conv shapes (C = per-pixel operand width)
    CONVS = [(f[0], *map(int, f[1:])) for f in (t.split(",") for t in os.environ["KB_CONVS"].split(";"))]
if os.environ.get("KB_HEADS"):  # the split-precision (3C-wide operand) head convs at 8 views
    CONVS = [("l1rn@148", V, 148, 148, 288, 256), ("l2rn@74", V, 74, 74, 576, 256), ("l3rn@37", V, 37, 37, 1152, 256),
             ("l4rn@19", V, 19, 19, 2304, 256), ("rn4@19", V, 19, 19, 768, 256), ("rn3@37", V, 37, 37, 768, 256),
             ("rn2@74", V, 74, 74, 768, 256), ("rn1@148", V, 148, 148, 768, 256), ("reg1@296", V, 296, 296, 768, 128),
             ("reg2@518", V, 518, 518, 384, 128), ("ip3s2@37", V, 37, 37, 2304, 768, 2)]
if ONLY:
    CONVS = [c for c in CONVS if c[0] in ONLY.split(",")]


ROUNDS = int(os.environ.get("KB_ROUNDS", "1"))
KBLOCKS = [int(v) for v in os.environ.get("KB_KBLOCK", "0").split(",")]


def interleaved(fns, reps):
    """Median time of each fn over KB_ROUNDS rounds, the fns interleaved inside every round (the guide's rule: A/B
    in one process, interleaved, so clock drift and the first-run penalty hit every variant alike)."""
    ts = [[] for _ in fns]
    for _ in range(ROUNDS):
        for i, f in enumerate(fns):
            ts[i].append(timeit(f, reps))
    return [sorted(t)[len(t) // 2] for t in ts]


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
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dt = torch.float16 if os.environ.get("KB_F16") else torch.bfloat16  # KB_F16=1: binary16 operands (the TF32 heads)
    if what in ("gemm", "all"):
        for name, M, N, K in GEMMS:
            A = (torch.randn(M, K, device="cuda") * 0.5).to(dt)
            W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(dt)
            b = torch.randn(N, device="cuda")
            o = torch.empty(M, N, device="cuda", dtype=dt)
            # the residual linears (attn proj, fc2) update the fp32 stream in place: x = x + gamma * (A W^T + b)
            resid = name.endswith(("proj", "fc2")) and not os.environ.get("KB_NO_RESID")
            x = torch.randn(M, N, device="cuda") if resid else None
            gam = torch.randn(N, device="cuda") * 0.1 if resid else None
            gelu = name.endswith("fc1") and not os.environ.get("KB_NO_RESID")  # the MLP's first linear: GELU epilogue
            # KB_LN=1: the residual linears with the next sub-block's LayerNorm fused (mapa_gemm_desc.ln_*, bf16 out)
            lnargs = None
            if resid and os.environ.get("KB_LN"):
                lnargs = (torch.randn(N, device="cuda"), torch.randn(N, device="cuda"), 1e-6,
                          torch.empty(M, N, device="cuda", dtype=dt))

            def run(var, gm=0):
                def f():
                    nat.gemm_set_variant(var)
                    nat.gemm_tune(nat.TUNE_TILE_GROUP, gm)
                    if resid and lnargs is not None:
                        nat.gemm(A, W, M, N, K, bias=b, gamma=gam, resid1=x, out_f32=x, ln=lnargs)
                    elif resid:
                        nat.gemm(A, W, M, N, K, bias=b, gamma=gam, resid1=x, out_f32=x)
                    elif gelu:
                        nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_lp=o)
                    else:
                        nat.gemm(A, W, M, N, K, bias=b, out_lp=o)
                return f
            combos = [(v, g) for v in VARIANTS for g in GMS]
            fns = [run(v, g) for v, g in combos]
            if "torch" in sys.argv:
                fns.append(lambda: torch.nn.functional.linear(A, W, b.to(dt)))
            mss = interleaved(fns, reps)
            for (var, gm), ms in zip(combos, mss):
                tag = f" gm{gm}" if len(GMS) > 1 else ""
                print(f"gemm {name:10s} v{var:<4d}{tag} M={M} N={N} K={K}: {ms*1e3:8.1f} us  {2*M*N*K/ms/1e9:7.1f} TF/s",
                      flush=True)
            nat.gemm_tune(nat.TUNE_TILE_GROUP, 0)
            if "torch" in sys.argv:
                print(f"gemm {name:10s} hipBLASLt via torch: {mss[-1]*1e3:8.1f} us  {2*M*N*K/mss[-1]/1e9:7.1f} TF/s",
                      flush=True)
            nat.gemm_set_variant(0)
    if what in ("conv", "all"):
        for name, n, H, W_, C, Co, *st in CONVS:  # optional 7th field: stride
            stride = st[0] if st else 1
            OH, OW = (H - 1) // stride + 1, (W_ - 1) // stride + 1
            # KB_SPLIT=1: C is the logical [hi | hi | lo] width of a split-precision operand (the fp32-exact heads):
            # the stored operand is [hi | lo] (2C/3 per pixel) and the weight is tagged as split-packed
            split = bool(os.environ.get("KB_SPLIT")) and C % 3 == 0 and (C // 3) % 32 == 0
            x = (torch.randn(n, H, W_, 2 * C // 3 if split else C, device="cuda") * 0.5).to(dt)
            w0 = (torch.randn(Co, 9 * C, device="cuda") * (9 * C) ** -0.5).to(dt)
            b = torch.randn(Co, device="cuda")
            o = torch.empty(n * OH * OW, Co, device="cuda", dtype=dt)
            M = n * OH * OW
            combos = []
            for kb in KBLOCKS:  # channel-block-major K order (mapa_gemm_desc.conv_kblock)
                w = w0
                if kb and C % kb == 0:
                    w = w0.view(Co, 9, C // kb, kb).permute(0, 2, 1, 3).contiguous().reshape(Co, -1)
                    w._mapa_kblock = kb
                if split:
                    w._mapa_split = True
                combos += [(var, kb, w) for var in VARIANTS]

            def runc(var, w):
                def f():
                    nat.gemm_set_variant(var)
                    nat.gemm(x, w, M, Co, 9 * C, bias=b, out_lp=o, conv=(C, H, W_, OH, OW, stride))
                return f
            for (var, kb, _), ms in zip(combos, interleaved([runc(v, w) for v, _, w in combos], reps)):
                print(f"conv {name:10s} v{var:<4d} kb{kb:<3d} M={M} N={Co} K={9*C}: {ms*1e3:8.1f} us  "
                      f"{2*M*Co*9*C/ms/1e9:7.1f} TF/s", flush=True)
            nat.gemm_set_variant(0)
    if what == "ln":  # the path's LayerNorms: fp32 residual rows -> bf16 GEMM operand
        for name, rows, dim in (("enc", R, 1024), ("aat", L - 1, 768)):
            x = torch.randn(rows, dim, device="cuda")
            w, b = torch.randn(dim, device="cuda"), torch.randn(dim, device="cuda")
            y = torch.empty(rows, dim, device="cuda", dtype=torch.bfloat16)
            f = lambda: nat.layernorm(x, rows, dim, w, b, y_lp=y)  # noqa: E731
            ms = timeit(f, reps)
            print(f"ln {name:6s} rows={rows} dim={dim}: {ms*1e3:7.1f} us  {rows*dim*6/ms/1e9:6.2f} TB/s", flush=True)
    if what == "bil":  # the DPT resizes: 2x align_corners upsamples and the regressor's 296^2 -> 518^2 split resize
        cases = [("up148", 74, 74, 148, 256, torch.float32, torch.float32),
                 ("up296s3", 148, 148, 296, 256, torch.float32, "s3"),
                 ("reg518", 296, 296, 518, 128, torch.float32, "s3")]
        for name, IH, IW, O, C, ti, to in cases:
            x = torch.randn(V, IH, IW, C, device="cuda", dtype=ti)
            o = torch.empty(V, O, O, 2 * C if to == "s3" else C, device="cuda",
                            dtype=torch.bfloat16 if to == "s3" else to)
            f = lambda: nat.bilinear_ac(x, V, IH, IW, C, O, O, O, O, o, split_out=(to == "s3"))  # noqa: E731
            ms = timeit(f, reps)
            nbytes = x.numel() * x.element_size() + o.numel() * o.element_size()
            print(f"bil {name:8s} {IH}->{O} C={C}: {ms*1e3:8.1f} us  {nbytes/ms/1e9:6.2f} TB/s (in + out once)", flush=True)
    if what in ("attn", "all"):
        cases = [("enc", V, 16, T + 1), ("frame", V, 12, T), ("global", 1, 12, L)]
        if os.environ.get("KB_ATTN_WIDE"):
            cases += [("global1", 1, 12, T + 1), ("global32", 1, 12, 32 * T + 1)]
        kvm = int(os.environ.get("KB_ATTN_KVMUL", "1"))  # seq_kv = kvm * seq_q (per-task overhead vs per-tile cost)
        for name, B, Hh, S in cases:
            C = Hh * 64
            qkv = torch.randn(B * S * kvm, 3 * C, device="cuda").to(dt)
            o = torch.empty(B * S, C, device="cuda", dtype=dt)
            rs = 3 * C
            Skv = S * kvm

            def mk():
                def f():
                    nat.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B, heads=Hh, seq_q=S, seq_kv=Skv,
                                  q_bstride=Skv * rs, q_rstride=rs, k_bstride=Skv * rs, k_rstride=rs,
                                  v_bstride=Skv * rs, v_rstride=rs, o_bstride=S * C, o_rstride=C)
                return f
            fns = [mk()]
            if os.environ.get("KB_ATTN_HM"):  # head-major [B*H][S][64] q / k / v (contiguous 128-B key rows)
                qh = torch.randn(B * Hh, S, 64, device="cuda").to(dt)
                kh = torch.randn(B * Hh, Skv, 64, device="cuda").to(dt)
                vh = torch.randn(B * Hh, Skv, 64, device="cuda").to(dt)
                oh = torch.empty(B * Hh, S, 64, device="cuda", dtype=dt)
                fns.append(lambda: nat.attention(qh, kh, vh, oh, batch=B * Hh, heads=1, seq_q=S, seq_kv=Skv,
                                                 q_bstride=S * 64, q_rstride=64, k_bstride=Skv * 64, k_rstride=64,
                                                 v_bstride=Skv * 64, v_rstride=64, o_bstride=S * 64, o_rstride=64))
            mss = interleaved(fns, reps)
            if os.environ.get("KB_ATTN_HM"):
                print(f"attn {name:10s} head-major kv x{kvm}: {mss[-1]*1e3:8.1f} us  "
                      f"{4*B*Hh*S*Skv*64/mss[-1]/1e9:7.1f} TF/s", flush=True)
                mss = mss[:-1]
            ms = mss[0]
            S2 = S * Skv
            if "torch" in sys.argv:
                t = qkv.view(B, S, 3, Hh, 64).permute(2, 0, 3, 1, 4)
                q, k, v = t[0].contiguous(), t[1].contiguous(), t[2].contiguous()
                ms_t = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v), reps)
                print(f"  torch SDPA {name}: {4*B*Hh*S*S*64/ms_t/1e9:7.1f} TF/s", flush=True)
            print(f"attn {name:10s} B={B} H={Hh} S={S} kv x{kvm}: {ms*1e3:8.1f} us  {4*B*Hh*S2*64/ms/1e9:7.1f} TF/s",
                  flush=True)


if __name__ == "__main__":
    main()

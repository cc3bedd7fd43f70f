"""Diagnostic: the bf16-output GELU epilogue against torch's exact GELU of the same pre-activation; prints the
worst elements by the tolerance ratio."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mapanything import _native as nat  # noqa: E402

torch.manual_seed(0)
M, N, K = 2741, 3072, 768
A = (torch.randn(M, K, device="cuda") * 1.5).to(torch.bfloat16)
W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
b = torch.randn(N, device="cuda")
for var in (0, 2570, 2571, 2574):
    pre = torch.empty(M, N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nat.gemm_set_variant(var)
    nat.gemm(A, W, M, N, K, bias=b, out_f32=pre)
    nat.gemm(A, W, M, N, K, bias=b, act=nat.ACT_GELU, out_lp=out)
    torch.cuda.synchronize()
    ref = F.gelu(pre.double())
    err = (out.double() - ref).abs()
    ratio = err / (ref.abs() * 2.0 ** -8 + 1e-30)
    v, i = ratio.flatten().topk(5)
    print(f"variant {var}: max ratio {float(v[0]):.3g}, flips {(out != ref.float().to(torch.bfloat16)).float().mean().item():.2e}")
    for r, j in zip(v.tolist(), i.tolist()):
        print(f"   ratio {r:.3g} pre {pre.flatten()[j].item():.9g} out {out.flatten()[j].item():.9g} ref {ref.flatten()[j].item():.9g}")
nat.gemm_set_variant(0)

"""Per-task fixed cost of the attention kernel: time at a fixed task count (8 x 16 heads x 11 query blocks, the
encoder layer) for growing key counts; the intercept of time vs key tiles is the per-wave-of-tasks overhead."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402


def timeit(fn, reps=30):
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


B, H, Sq = 8, 16, 1370
C = H * 64
for Skv in (64, 128, 256, 512, 1370, 2740):
    q = torch.randn(B * Sq, C, device="cuda").to(torch.bfloat16)
    kv = torch.randn(B * Skv, 2 * C, device="cuda").to(torch.bfloat16)
    o = torch.empty(B * Sq, C, device="cuda", dtype=torch.bfloat16)
    f = lambda: nat.attention(q, kv, kv[:, C:], o, batch=B, heads=H, seq_q=Sq, seq_kv=Skv,  # noqa: E731
                              q_bstride=Sq * C, q_rstride=C, k_bstride=Skv * 2 * C, k_rstride=2 * C,
                              v_bstride=Skv * 2 * C, v_rstride=2 * C, o_bstride=Sq * C, o_rstride=C)
    us = timeit(f)
    print(f"Skv={Skv:6d} tiles={(Skv + 63) // 64:4d}: {us:8.1f} us  {4 * B * H * Sq * Skv * 64 / us / 1e6:7.1f} TF/s",
          flush=True)

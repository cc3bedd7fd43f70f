"""Attention throughput across sequence lengths at a fixed total of query rows (per-task overhead vs steady state):
python tools/attn_sweep.py.  Times each shape with HIP events over 20 launches after 3 warm-ups."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

if os.environ.get("MAPA_AB_LIB"):
    nat.load_library(os.environ["MAPA_AB_LIB"])


def run(B, Hh, S, reps=20):
    C = Hh * 64
    qkv = torch.randn(B * S, 3 * C, device="cuda").to(torch.bfloat16)
    o = torch.empty(B * S, C, device="cuda", dtype=torch.bfloat16)
    rs = 3 * C

    def once():
        nat.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B, heads=Hh, seq_q=S, seq_kv=S, q_bstride=S * rs,
                      q_rstride=rs, k_bstride=S * rs, k_rstride=rs, v_bstride=S * rs, v_rstride=rs,
                      o_bstride=S * C, o_rstride=C)
    for _ in range(3):
        once()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        once()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    fl = 4.0 * B * Hh * S * S * 64
    print(f"B={B:3d} H={Hh:2d} S={S:6d}  {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)


shapes = [(8, 16, 1370), (8, 12, 1369), (4, 16, 2740), (1, 16, 10960), (1, 12, 10953), (8, 16, 1280), (8, 16, 1408),
          (8, 16, 1536)]
if len(sys.argv) > 1:  # "B,H,S B,H,S ..."
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for shape in shapes:
    run(*shape)

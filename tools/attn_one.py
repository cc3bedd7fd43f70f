"""One attention shape, N launches (for rocprofv3 PMC passes): python tools/attn_one.py [B H S reps]."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

if os.environ.get("MAPA_AB_LIB"):  # A/B builds: load before any other call
    nat.load_library(os.environ["MAPA_AB_LIB"])

B, Hh, S, reps = (int(x) for x in (sys.argv[1:5] if len(sys.argv) >= 5 else (1, 12, 8 * 1369 + 1, 10)))
C = Hh * 64
qkv = torch.randn(B * S, 3 * C, device="cuda").to(torch.bfloat16)
o = torch.empty(B * S, C, device="cuda", dtype=torch.bfloat16)
rs = 3 * C
for _ in range(reps):
    nat.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, batch=B, heads=Hh, seq_q=S, seq_kv=S, q_bstride=S * rs,
                  q_rstride=rs, k_bstride=S * rs, k_rstride=rs, v_bstride=S * rs, v_rstride=rs, o_bstride=S * C,
                  o_rstride=C)
torch.cuda.synchronize()
print("ok")

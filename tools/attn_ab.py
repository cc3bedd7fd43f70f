"""Attention kernel A/B (one arm per process, MAPA_ATTN_PP picks the kernel): the path's three attention shapes
(encoder 8 x 16 x 1370, frame 8 x 12 x 1369, global 1 x 12 x (8*1369+1); bf16, qkv packed as the engine lays it
out), seeded inputs, HIP-event time per launch (median of 3 runs of `reps`) and a SHA-256 of every output (bitwise
comparison across arms).  Usage: MAPA_ATTN_PP=1 python tools/attn_ab.py [reps] >> gpurun_out/attn_ab.jsonl"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

if os.environ.get("MAPA_AB_LIB"):  # A/B builds (tools/ab_build.sh): load before any other call
    nat.load_library(os.environ["MAPA_AB_LIB"])

SHAPES = [("encoder", 8, 16, 1370), ("frame", 8, 12, 1369), ("global", 1, 12, 8 * 1369 + 1)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    res = {"arm": os.environ.get("AB_ARM", os.environ.get("MAPA_ATTN_PP", "0"))}
    for name, B, H, S in SHAPES:
        C = H * 64
        g = torch.Generator(device="cuda").manual_seed(1234 + S)
        qkv = (torch.randn(B * S, 3 * C, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
        o = torch.empty(B * S, C, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * H * S, device="cuda", dtype=torch.float32)
        rs = 3 * C

        def f():
            kw = dict(batch=B, heads=H, seq_q=S, seq_kv=S, q_bstride=S * rs, q_rstride=rs, k_bstride=S * rs,
                      k_rstride=rs, v_bstride=S * rs, v_rstride=rs, o_bstride=S * C, o_rstride=C, lse=lse)
            nat.attention(qkv, qkv[:, C:], qkv[:, 2 * C:], o, **kw)

        for _ in range(3):
            f()
        ts = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(reps):
                f()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / reps * 1e3)
        us = sorted(ts)[1]
        flop = 4.0 * B * H * S * S * 64
        res[name] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1),
                     "sha_o": hashlib.sha256(o.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16],
                     "sha_lse": hashlib.sha256(lse.cpu().numpy().tobytes()).hexdigest()[:16]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

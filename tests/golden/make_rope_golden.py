"""Fixtures for RoPE-2D from the REAL reference (run in the build container only):

    python tests/golden/make_rope_golden.py     # writes tests/golden/golden_rope2d.npz

Imports uniception.models.libs.croco.pos_embed from /root/reference through ref_harness (stubbed non-arithmetic
imports).  Its cuRoPE2D extension is not built there, so `RoPE2D` is the pure-torch class of pos_embed.py:108-155
(the same rotation as curope/kernels.cu:17-82).  Saved: seeded fp32 tokens, int64 positions, and the reference's
output, for (a) a 37x37 patch grid (PositionGetter's cartesian_prod(y, x) order) with 2 heads of 64 and
(b) random positions up to 300 with 3 heads of 64 and two batch elements (base 100 and base 10000).
"""

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402


def main():
    ref_harness.install_stubs()
    if ref_harness.REF not in sys.path:
        sys.path.insert(0, ref_harness.REF)
    from uniception.models.libs.croco import pos_embed

    RoPE2D = pos_embed.RoPE2D
    assert RoPE2D.__name__ == "RoPE2D" and hasattr(RoPE2D, "apply_rope1d"), "expected the pure-torch RoPE2D"
    g = torch.Generator().manual_seed(2024)
    out = {}
    # (a) one view's 37 x 37 grid, 2 heads x 64
    h = w = 37
    pos = torch.cartesian_prod(torch.arange(h), torch.arange(w)).view(1, h * w, 2)
    tok = torch.randn(1, 2, h * w, 64, generator=g)
    out["grid_tokens"], out["grid_pos"] = tok.numpy(), pos.numpy()
    out["grid_out"] = RoPE2D(freq=100.0)(tok.clone(), pos).numpy()
    # (b) random positions, 2 batch elements, 3 heads; two bases
    pos = torch.randint(0, 300, (2, 200, 2), generator=g)
    tok = torch.randn(2, 3, 200, 64, generator=g)
    out["rand_tokens"], out["rand_pos"] = tok.numpy(), pos.numpy()
    out["rand_out_base100"] = RoPE2D(freq=100.0)(tok.clone(), pos).numpy()
    out["rand_out_base10000"] = RoPE2D(freq=10000.0)(tok.clone(), pos).numpy()
    np.savez_compressed(os.path.join(HERE, "golden_rope2d.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()

"""RoPE-2D of uniception's croco library (uniception/models/libs/croco/pos_embed.py:101-155 and its CUDA twin
curope/curope2d.py + kernels.cu:17-82) on MI355X: the rotation runs in the gfx950 kernel `mapa_rope2d`
(include/mapa.h), in place on the caller's tensor as cuRoPE2D does.  No CPU path: a missing library or device
raises (mapanything._native).

    rope = RoPE2D(freq=100.0, F0=1.0)
    q = rope(q, positions)     # q (B, heads, N, D) bf16/fp32 on the GPU, positions (B, N, 2) int64 (y, x)
"""

import torch

from mapanything import _native as nat


class RoPE2D:
    """Same constructor and forward contract as the reference's RoPE2D / cuRoPE2D (pos_embed.py:109-155,
    curope2d.py:31-40): tokens (B, H, N, D) with D % 16 == 0 (the reference asserts D % 2; the kernel's 4-wide
    lanes need D/4 % 4 == 0, true for every head width the models use), positions (B, N, 2) integer (y, x).
    The rotation is applied in place (the head dim must be contiguous) and the tensor is returned."""

    def __init__(self, freq: float = 100.0, F0: float = 1.0):
        self.base = float(freq)
        self.F0 = float(F0)

    def __call__(self, tokens: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        return self.forward(tokens, positions)

    def forward(self, tokens: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        assert tokens.size(3) % 2 == 0, "number of dimensions should be a multiple of two"
        assert positions.ndim == 3 and positions.shape[-1] == 2  # Batch, Seq, 2
        B, H, N, D = tokens.shape
        if positions.shape[:2] != (B, N):
            raise ValueError(f"positions {tuple(positions.shape)} do not match tokens (B={B}, N={N})")
        if tokens.stride(3) != 1:
            raise ValueError("RoPE2D: the head dimension must be contiguous")
        pos = positions.to(device=tokens.device, dtype=torch.int64).contiguous()
        nat.rope2d(tokens, pos, B, H, N, D, tokens.stride(0), tokens.stride(1), tokens.stride(2), self.base, self.F0)
        return tokens


cuRoPE2D = RoPE2D  # curope2d.py:31: the CUDA class the reference prefers when its extension is built

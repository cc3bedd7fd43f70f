"""Deterministic synthetic checkpoints and inputs (no network, no released weights here).

There is no MapAnything checkpoint in this environment, so every parity test and every
benchmark runs on a *named-tensor PRNG* checkpoint: each tensor of the state dict is filled from a
counter-based splitmix64 stream whose seed is the FNV-1a hash of the tensor's state-dict name.  The same
bytes are produced by this numpy implementation on any host, so the fixture generator (which loads them
into the reference `MapAnything`, model.py:96), the CPU oracle and the HIP engine all see identical weights.

Scale classes follow the roles of the tensors in the reference modules:
  * Linear / Conv2d weights (out, in, ...):        U(-a, a), a = sqrt(3 / fan_in)   (unit-variance gain)
  * ConvTranspose2d weights (in, out, kh, kw):      fan_in = in   (dpt.py input_process.{0,1}.0.1)
  * biases:                                        U(-0.02, 0.02)
  * LayerNorm weight / bias:                       1 + U(-0.1, 0.1) / U(-0.05, 0.05)
  * DINOv2 LayerScale gamma (layers/layer_scale.py): 0.1 + U(-0.02, 0.02)  (trained-magnitude mimic)
  * pos_embed / cls_token / scale_token:           U(-0.03, 0.03)
  * AAT view_pos_table buffer:                     the reference's sinusoid table (alternating_attention_transformer.py:189-198)
"""

from __future__ import annotations

import math
from typing import Dict, Iterable, List, Tuple

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
GLOBAL_SEED = 0x5EED_0F_3D_4A_11


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix_uniform(seed: int, n: int) -> np.ndarray:
    """n float32 values in [0, 1): u_i = (splitmix64(seed + (i+1)*golden) >> 40) * 2^-24 (exact in fp32)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        x = np.uint64(seed) + idx * _GOLDEN
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return (x >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)


def named_uniform(name: str, shape: Tuple[int, ...], lo: float, hi: float, seed: int = GLOBAL_SEED) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = splitmix_uniform(fnv1a64(name) ^ seed, n)
    t = u * np.float32(2.0) - np.float32(1.0)                        # exact: [-1, 1)
    half = np.float32((hi - lo) / 2.0)
    mid = np.float32((hi + lo) / 2.0)
    return (t * half + mid).astype(np.float32).reshape(shape)


def sinusoid_table(n_position: int, d_hid: int, base: float = 10000.0) -> np.ndarray:
    """Restates alternating_attention_transformer.py:189-198 (float64 table cast to float32)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)
    angle = pos / np.power(base, 2 * (j // 2) / d_hid)
    angle[:, 0::2] = np.sin(angle[:, 0::2])
    angle[:, 1::2] = np.cos(angle[:, 1::2])
    return angle.astype(np.float32)


CONV_TRANSPOSE_WEIGHTS = (
    "dpt_feature_head.input_process.0.0.1.weight",
    "dpt_feature_head.input_process.1.0.1.weight",
)


def tensor_init(name: str, shape: Tuple[int, ...]) -> np.ndarray:
    """Synthetic value of one state-dict entry (see module docstring for the classes)."""
    if name.endswith("view_pos_table"):
        return sinusoid_table(shape[0], shape[1])
    leaf = name.rsplit(".", 1)[-1]
    if leaf in ("pos_embed", "cls_token") or name == "scale_token" or name.endswith(".scale_token"):
        return named_uniform(name, shape, -0.03, 0.03)
    if leaf == "gamma":
        return named_uniform(name, shape, 0.08, 0.12)
    if len(shape) >= 2 and leaf == "weight":
        if any(name.endswith(c) for c in CONV_TRANSPOSE_WEIGHTS):
            fan_in = shape[0]
        else:
            fan_in = int(np.prod(shape[1:]))
        a = math.sqrt(3.0 / fan_in)
        return named_uniform(name, shape, -a, a)
    if len(shape) == 1 and leaf == "weight":  # LayerNorm
        return named_uniform(name, shape, 0.9, 1.1)
    if leaf == "bias":
        parent = name.rsplit(".", 2)[-2] if name.count(".") >= 1 else ""
        if "norm" in parent:
            return named_uniform(name, shape, -0.05, 0.05)
        return named_uniform(name, shape, -0.02, 0.02)
    raise KeyError(f"no synthetic init rule for {name} {shape}")


def synthetic_state_dict(spec: Iterable[Tuple[str, Tuple[int, ...]]]) -> Dict[str, np.ndarray]:
    return {name: tensor_init(name, tuple(shape)) for name, shape in spec}


# ----------------------------------------------------------------------------------------------------------
# Inputs: uint8-uniform images -> /255 -> DINOv2 mean/std (image_normalizations.py:21)
# ----------------------------------------------------------------------------------------------------------
DINOV2_MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
DINOV2_STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def synthetic_images(num_views: int, height: int, width: int, seed: int, batch: int = 1) -> List[np.ndarray]:
    """num_views arrays (batch, 3, H, W) float32, DINOv2-normalised, from the named PRNG."""
    out = []
    for v in range(num_views):
        u = splitmix_uniform(fnv1a64(f"image/{seed}/{v}") ^ GLOBAL_SEED, batch * 3 * height * width)
        px = np.floor(u * np.float32(256.0)).astype(np.float32) / np.float32(255.0)
        px = px.reshape(batch, 3, height, width)
        out.append(((px - DINOV2_MEAN[None, :, None, None]) / DINOV2_STD[None, :, None, None]).astype(np.float32))
    return out


def synthetic_intrinsics(num_views: int, height: int, width: int, seed: int, batch: int = 1) -> List[np.ndarray]:
    """fx=fy=0.8*W*(1 +- 5 %), cx=W/2, cy=H/2."""
    out = []
    for v in range(num_views):
        u = splitmix_uniform(fnv1a64(f"intrinsics/{seed}/{v}") ^ GLOBAL_SEED, batch)
        f = np.float32(0.8 * width) * (np.float32(0.95) + np.float32(0.1) * u)
        K = np.zeros((batch, 3, 3), dtype=np.float32)
        K[:, 0, 0] = f
        K[:, 1, 1] = f
        K[:, 0, 2] = width / 2.0
        K[:, 1, 2] = height / 2.0
        K[:, 2, 2] = 1.0
        out.append(K)
    return out


def synthetic_poses(num_views: int, seed: int, batch: int = 1) -> List[np.ndarray]:
    """cam2world 4x4 poses: rotation from a normalised uniform quaternion, translation in U[-2, 2] m."""
    out = []
    for v in range(num_views):
        u = splitmix_uniform(fnv1a64(f"pose/{seed}/{v}") ^ GLOBAL_SEED, batch * 7).reshape(batch, 7)
        q = (2.0 * u[:, :4] - 1.0).astype(np.float64)
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
        P = np.zeros((batch, 4, 4), dtype=np.float64)
        P[:, 0] = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y), 4 * u[:, 4] - 2], 1)
        P[:, 1] = np.stack([2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x), 4 * u[:, 5] - 2], 1)
        P[:, 2] = np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y), 4 * u[:, 6] - 2], 1)
        P[:, 3, 3] = 1.0
        out.append(P.astype(np.float32))
    return out


def synthetic_sparse_depth(num_views: int, height: int, width: int, seed: int, keep: float = 0.1,
                           batch: int = 1) -> List[np.ndarray]:
    """depth_z in U[0.5, 10] m with (1-keep) of the pixels zeroed."""
    out = []
    for v in range(num_views):
        u = splitmix_uniform(fnv1a64(f"depth/{seed}/{v}") ^ GLOBAL_SEED, batch * height * width)
        m = splitmix_uniform(fnv1a64(f"depthmask/{seed}/{v}") ^ GLOBAL_SEED, batch * height * width)
        d = (np.float32(0.5) + np.float32(9.5) * u) * (m < np.float32(keep)).astype(np.float32)
        out.append(d.reshape(batch, height, width).astype(np.float32))
    return out

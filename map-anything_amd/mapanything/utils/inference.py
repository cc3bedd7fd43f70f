"""infer() host glue: input validation / preprocessing (reference mapanything/utils/inference.py:130-311) and
output post-processing (inference.py:314-506) with the per-pixel work in HIP kernels (postprocess.hip)."""

from __future__ import annotations

import functools
from typing import Any, Dict, List

import numpy as np
import torch

from .. import _native as nat

ALLOWED_VIEW_KEYS = {
    "img", "data_norm_type", "intrinsics", "ray_directions", "depth_z", "camera_poses", "is_metric_scale",
    "instance", "idx", "true_shape",
}
REQUIRED_KEYS = {"data_norm_type"}
CONFLICTING_KEYS = [("intrinsics", "ray_directions")]


def validate_input_views_for_inference(views: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    """inference.py:130-219 (same checks, same ValueError messages)."""
    if not views:
        raise ValueError("At least one view must be provided")
    views_with_poses = []
    for view_idx, view in enumerate(views):
        provided = set(view.keys())
        missing = REQUIRED_KEYS - provided
        if missing:
            raise ValueError(f"View {view_idx} missing required keys: {missing}")
        for conflict_set in CONFLICTING_KEYS:
            present = [k for k in conflict_set if k in provided]
            if len(present) > 1:
                raise ValueError(f"View {view_idx} contains conflicting keys: {present}. "
                                 f"Only one of {conflict_set} can be provided at a time.")
        if view_idx == 0 and "img" not in provided:
            raise ValueError("The First View missing required keys: img")
        if "img" not in provided:
            if "intrinsics" not in provided and "ray_directions" not in provided:
                raise ValueError(f"View {view_idx} without image must provide intrinsics or ray_directions")
            if "camera_poses" not in provided:
                raise ValueError(f"View {view_idx} without image must provide camera_poses")
        if "depth_z" in provided and "intrinsics" not in provided and "ray_directions" not in provided:
            raise ValueError(
                f"View {view_idx} depth constraint violation: If 'depth_z' is provided, then 'intrinsics' or "
                f"'ray_directions' must also be provided. Z Depth values require camera calibration information "
                f"to be meaningful for an image.")
        if "camera_poses" in provided:
            views_with_poses.append(view_idx)
    if views_with_poses and 0 not in views_with_poses:
        raise ValueError(
            f"Camera pose constraint violation: Views {views_with_poses} have camera_poses, but view 0 (reference "
            f"view) does not. When using camera_poses, the first view must also provide camera_poses to serve as "
            f"the reference frame.")
    return views


def get_rays_in_camera_frame(intrinsics: torch.Tensor, height: int, width: int) -> torch.Tensor:
    """geometry.py:186-241 (unit-sphere normalised ray directions, (B,H,W,3)) — mapa_view_rays kernel."""
    K = intrinsics.to(torch.float32).contiguous()
    B = K.shape[0]
    rays = torch.empty(B, height, width, 3, device=K.device, dtype=torch.float32)
    nat.view_rays(B, height, width, rays, K=K)
    return rays


def preprocess_input_views_for_inference(views: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    """inference.py:222-311.  Per-pixel work (rays from intrinsics or renormalised rays, depth_z -> depth along
    the ray) in one mapa_view_rays launch per view; the per-view 3x3 -> quaternion stays a small tensor op."""
    out = []
    for view in views:
        pv = dict(view)
        if "intrinsics" in view or "ray_directions" in view:
            H, W = view["img"].shape[-2:]
            dev = view["img"].device
            B = view["img"].shape[0]
            rays = torch.empty(B, H, W, 3, device=dev, dtype=torch.float32)
            dz = view["depth_z"].to(torch.float32).contiguous() if "depth_z" in view else None
            dar = torch.empty(B, H, W, 1, device=dev, dtype=torch.float32) if dz is not None else None
            if "intrinsics" in view:
                nat.view_rays(B, H, W, rays, K=view["intrinsics"].to(torch.float32).contiguous(), depth_z=dz,
                              depth_along_ray=dar)
                del pv["intrinsics"]
            else:
                nat.view_rays(B, H, W, rays, rays_in=view["ray_directions"].to(torch.float32).contiguous(),
                              depth_z=dz, depth_along_ray=dar)
            pv["ray_directions"] = rays
            if dz is not None:
                pv["depth_along_ray"] = dar
                del pv["depth_z"]
        if "camera_poses" in view:
            cp = view["camera_poses"]
            if isinstance(cp, tuple) and len(cp) == 2:
                pv["camera_pose_quats"], pv["camera_pose_trans"] = cp
            elif torch.is_tensor(cp) and cp.shape[-2:] == (4, 4):
                pv["camera_pose_quats"] = rotation_matrix_to_quaternion(cp[:, :3, :3])
                pv["camera_pose_trans"] = cp[:, :3, 3]
            else:
                raise ValueError("camera_poses must be either a tuple of (quats, trans) or a tensor of (B, 4, 4) "
                                 "transformation matrices.")
            del pv["camera_poses"]
        if "is_metric_scale" not in pv:
            pv["is_metric_scale"] = torch.ones(view["img"].shape[0], dtype=torch.bool)  # host flag, read on host
        if "ray_directions" in pv:
            pv["ray_directions_cam"] = pv.pop("ray_directions")
        out.append(pv)
    return out


def rotation_matrix_to_quaternion(m: torch.Tensor) -> torch.Tensor:
    """geometry.py:655-713 (xyzw, w >= 0)."""
    import torch.nn.functional as F

    bd = m.shape[:-2]
    m00, m01, m02, m10, m11, m12, m20, m21, m22 = torch.unbind(m.reshape(bd + (9,)), -1)
    qa = torch.stack([1 + m00 + m11 + m22, 1 + m00 - m11 - m22, 1 - m00 + m11 - m22, 1 - m00 - m11 + m22], -1)
    qa = torch.where(qa > 0, torch.sqrt(torch.clamp(qa, min=0)), torch.zeros_like(qa))
    cand = torch.stack([
        torch.stack([qa[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], -1),
        torch.stack([m21 - m12, qa[..., 1] ** 2, m10 + m01, m02 + m20], -1),
        torch.stack([m02 - m20, m10 + m01, qa[..., 2] ** 2, m12 + m21], -1),
        torch.stack([m10 - m01, m20 + m02, m21 + m12, qa[..., 3] ** 2], -1)], -2)
    cand = cand / (2.0 * qa[..., None].max(torch.tensor(0.1, device=m.device)))
    out = cand[F.one_hot(qa.argmax(-1), 4) > 0.5, :].reshape(bd + (4,))[..., [1, 2, 3, 0]]
    return torch.where(out[..., 3:4] < 0, -out, out)


@functools.lru_cache(maxsize=64)
def normal_cos_threshold(tol_deg: float) -> float:
    """normals_edge compares numpy's float32 arccos of each window dot product with np.deg2rad(tol) in float64
    (geometry.py:2248-2258).  arccos is monotone, so that test is `dot < c` for one float32 boundary c: found here
    by bisection over the ordered float32 values in [-1, 1] with numpy's own float32 arccos (the function the
    reference calls), checked against the library's double-precision boundary and verified on the 1024 floats
    around it.  -1: no angle exceeds tol; 2: every angle does (also the 0 of masked-out entries)."""
    tol = np.deg2rad(tol_deg)

    def edge(d):
        return bool(np.float64(np.arccos(np.float32(d))) > tol)

    if not edge(-1.0):
        return -1.0
    if edge(1.0):
        return 2.0
    bits = lambda f: int(np.float32(f).view(np.int32))  # noqa: E731

    def key(f):  # order-preserving int of a float32
        b = bits(f)
        return b if b >= 0 else -(b & 0x7FFFFFFF)

    def unkey(k):
        b = k if k >= 0 else (-k) | -0x80000000
        return float(np.int32(b).view(np.float32))

    lo, hi = key(-1.0), key(1.0)
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if edge(unkey(mid)):
            lo = mid
        else:
            hi = mid
    cs = np.array([unkey(k) for k in range(hi - 512, hi + 512)], np.float32)
    cs = cs[(cs >= -1) & (cs <= 1)]
    assert np.array_equal(np.arccos(cs).astype(np.float64) > tol, cs < np.float32(unkey(hi))), \
        "numpy arccos is not monotone around the normal-edge threshold"
    return unkey(hi)


def postprocess_outputs(raw: Dict[str, torch.Tensor], imgs: torch.Tensor, mean: torch.Tensor, std: torch.Tensor, *,
                        apply_mask=True, mask_edges=True, edge_normal_threshold=5.0, edge_depth_threshold=0.03,
                        apply_confidence_mask=False, confidence_percentile=10) -> Dict[str, torch.Tensor]:
    """postprocess_model_outputs_for_inference (inference.py:314-506) on batched view-major tensors."""
    V, _, H, W = imgs.shape
    out = dict(raw)
    img_nn = torch.empty(V, H, W, 3, device=imgs.device, dtype=torch.float32)
    nat.denorm_image(imgs, V, H, W, mean, std, img_nn)
    out["img_no_norm"] = img_nn
    K = torch.empty(V, 3, 3, device=imgs.device, dtype=torch.float32)
    nat.recover_intrinsics(raw["ray_directions"], V, H, W, K)
    out["intrinsics"] = K
    if apply_mask:
        m_in = raw["non_ambiguous_mask"]
        if apply_confidence_mask:
            m_conf = torch.empty(V, H, W, device=imgs.device, dtype=torch.bool)
            nat.confidence_mask(raw["conf"], m_in, m_conf, V, H * W, confidence_percentile / 100.0)
            m_in = m_conf
        m_out = torch.empty(V, H, W, device=imgs.device, dtype=torch.bool)  # kernels write 0/1 bytes
        work = torch.empty(V * H * W * 17, device=imgs.device, dtype=torch.uint8) if mask_edges else None
        nat.postprocess_mask(raw["pts3d"], raw["pts3d_cam"], m_in, m_out, V, H, W,
                             normal_cos_threshold(float(edge_normal_threshold)), float(edge_depth_threshold),
                             bool(mask_edges), work)
        # zero the masked geometry in place (the raw tensors are this call's own outputs)
        nat.apply_mask(raw["pts3d"], raw["pts3d_cam"], raw["depth_along_ray"], m_out, V * H * W)
        out["mask"] = m_out
    return out

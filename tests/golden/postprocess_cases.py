"""Seeded raw-output scenes for the infer() post-processing fixtures (edge / normal / depth / confidence masks).

Shared by the fixture generator (make_postprocess_golden.py, which runs the reference's own
`postprocess_model_outputs_for_inference`, inference.py:314-506) and by the tests, which rebuild the same inputs
from the same seeds.  Pure numpy float32 arithmetic, so the inputs are identical on every machine.

A scene per view: unit pinhole rays, a depth field made of a slanted plane, a raised box (depth steps), a
crease (two planes meeting), a spherical bump, a high-frequency ripple patch and multiplicative noise; a few
zero-depth pixels and a few NaN points; camera-to-world pose applied for pts3d.  The non-ambiguous mask is mostly
true with rectangular holes, isolated false pixels and (in some views) a false border strip; one view of the
small case is entirely false (the reference's `batch_final_mask.any()` branch).  Confidences are quantised so
the percentile threshold meets ties.
"""

import numpy as np

CASES = {
    "pp_small": dict(views=3, h=48, w=64, seed=21),
    "pp_mid": dict(views=2, h=120, w=160, seed=23),
    "pp_518": dict(views=1, h=518, w=518, seed=22),
}

# infer() keyword sets exercised per case (inference.py:314-323 defaults: 5.0 deg, 0.03, conf off, 10 %)
OPTIONS = [
    dict(mask_edges=True, edge_normal_threshold=5.0, edge_depth_threshold=0.03, apply_confidence_mask=False,
         confidence_percentile=10),
    dict(mask_edges=True, edge_normal_threshold=5.0, edge_depth_threshold=0.03, apply_confidence_mask=True,
         confidence_percentile=25),
    dict(mask_edges=True, edge_normal_threshold=2.0, edge_depth_threshold=0.01, apply_confidence_mask=False,
         confidence_percentile=10),
    dict(mask_edges=True, edge_normal_threshold=30.0, edge_depth_threshold=0.2, apply_confidence_mask=True,
         confidence_percentile=10),
    dict(mask_edges=False, edge_normal_threshold=5.0, edge_depth_threshold=0.03, apply_confidence_mask=True,
         confidence_percentile=50),
]

MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)


def _rot(rng):
    a = rng.normal(size=3) * 0.3
    th = float(np.linalg.norm(a))
    k = a / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return (np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx).astype(np.float32)


def make_scene(case):
    """-> dict of float32/bool arrays with a leading view axis:
    pts3d, pts3d_cam (V,H,W,3), ray_directions (V,H,W,3), depth_along_ray (V,H,W,1), conf (V,H,W),
    non_ambiguous_mask (V,H,W) bool, img (V,3,H,W) DINOv2-normalised, cam_trans (V,3), cam_quats (V,4)."""
    V, H, W, seed = case["views"], case["h"], case["w"], case["seed"]
    rng = np.random.default_rng(seed)
    out = {k: [] for k in ("pts3d", "pts3d_cam", "ray_directions", "depth_along_ray", "conf",
                           "non_ambiguous_mask", "img", "cam_trans", "cam_quats")}
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    for v in range(V):
        f = np.float32(rng.uniform(0.7, 1.2) * W)
        cx, cy = np.float32(W / 2 + rng.uniform(-3, 3)), np.float32(H / 2 + rng.uniform(-3, 3))
        d = np.stack([(xx - cx) / f, (yy - cy) / f, np.ones_like(xx)], -1).astype(np.float32)
        rays = (d / np.linalg.norm(d, axis=-1, keepdims=True)).astype(np.float32)
        u, w_ = xx / np.float32(W), yy / np.float32(H)
        depth = (2.0 + 0.4 * u + 0.25 * w_).astype(np.float32)
        # raised box: depth steps on its border
        x0, y0 = rng.integers(0, W // 2), rng.integers(0, H // 2)
        box = (xx >= x0) & (xx < x0 + W // 3) & (yy >= y0) & (yy < y0 + H // 3)
        depth = np.where(box, depth - np.float32(rng.uniform(0.2, 0.6)), depth)
        # crease: a second plane folded in
        uc = np.float32(rng.uniform(0.55, 0.8))
        depth = depth + np.float32(1.5) * np.maximum(u - uc, 0)
        # spherical bump
        bx, by, br = rng.uniform(0.2, 0.8) * W, rng.uniform(0.2, 0.8) * H, rng.uniform(0.08, 0.2) * min(H, W)
        r2 = ((xx - bx) ** 2 + (yy - by) ** 2) / np.float32(br * br)
        depth = depth - np.where(r2 < 1, np.float32(0.3) * np.sqrt(np.maximum(1 - r2, 0)), 0).astype(np.float32)
        # high-frequency ripple patch (many normal edges)
        rp = (xx > W * 0.1) & (xx < W * 0.35) & (yy > H * 0.6) & (yy < H * 0.9)
        depth = np.where(rp, depth + np.float32(0.02) * np.sin(xx * 1.7) * np.cos(yy * 1.3), depth)
        depth = (depth * (1 + rng.normal(0, 2e-4, depth.shape))).astype(np.float32)
        # zero-depth pixels
        zero = rng.random((H, W)) < 0.01
        depth = np.where(zero, np.float32(0), depth).astype(np.float32)
        pts_cam = (rays * depth[..., None]).astype(np.float32)
        # a few NaN points
        nanpix = rng.random((H, W)) < 0.004
        pts_cam = np.where(nanpix[..., None], np.float32(np.nan), pts_cam).astype(np.float32)
        R, t = _rot(rng), rng.normal(size=3).astype(np.float32)
        pts = (pts_cam @ R.T + t).astype(np.float32)
        mask = np.ones((H, W), bool)
        for _ in range(3):
            hx, hy = rng.integers(0, W - 4), rng.integers(0, H - 4)
            mask[hy:hy + rng.integers(2, max(3, H // 6)), hx:hx + rng.integers(2, max(3, W // 6))] = False
        mask &= rng.random((H, W)) > 0.01
        if v % 2 == 1:
            mask[:, : max(1, W // 20)] = False
        if case["views"] == 3 and v == 2:
            mask[:] = False
        conf = (1.0 + np.round(rng.random((H, W)) * 40) / 8).astype(np.float32)
        img = ((rng.random((3, H, W)).astype(np.float32) - MEAN[:, None, None]) / STD[:, None, None]).astype(
            np.float32)
        q = rng.normal(size=4).astype(np.float32)
        q = (q / np.linalg.norm(q)).astype(np.float32)
        out["pts3d"].append(pts)
        out["pts3d_cam"].append(pts_cam)
        out["ray_directions"].append(rays)
        out["depth_along_ray"].append(np.linalg.norm(pts_cam, axis=-1, keepdims=True).astype(np.float32))
        out["conf"].append(conf)
        out["non_ambiguous_mask"].append(mask)
        out["img"].append(img)
        out["cam_trans"].append(t)
        out["cam_quats"].append(q)
    return {k: np.stack(v, 0) for k, v in out.items()}


def option_key(i):
    return f"opt{i}"

"""Shared helpers for the test-suite (no reference access: the released config is committed as a fixture)."""

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def released_config():
    """configs/inference.json of the reference (committed copy: tests/golden/inference_config.json)."""
    with open(os.path.join(HERE, "golden", "inference_config.json")) as f:
        return json.load(f)


# Golden cases (tests/golden/make_golden.py builds the same views for the reference)
CASES = {
    "cfg1_224": dict(views=2, h=224, w=224, seed=1),
    "v2_518": dict(views=2, h=518, w=518, seed=2),
    "mm_224": dict(views=2, h=224, w=224, seed=4, multimodal=True),
    "mixed_224": dict(views=3, h=224, w=224, seed=5, mixed=True),
    "ns_280x392": dict(views=2, h=280, w=392, seed=6),
    "one_224": dict(views=1, h=224, w=224, seed=7, rays_only=True),
}


def make_views(case):
    """Seeded reference-format views: images (+ intrinsics / sparse depth_z / 4x4 poses / is_metric_scale)."""
    import torch

    from mapanything.utils import synthetic

    n, h, w, seed = case["views"], case["h"], case["w"], case["seed"]
    imgs = synthetic.synthetic_images(n, h, w, seed)
    views = []
    for v in range(n):
        view = {"img": torch.from_numpy(imgs[v]), "data_norm_type": ["dinov2"]}
        if case.get("multimodal"):
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed)[v])
            view["depth_z"] = torch.from_numpy(synthetic.synthetic_sparse_depth(n, h, w, seed)[v])
            view["is_metric_scale"] = torch.ones(1, dtype=torch.bool)
        if case.get("rays_only"):
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed)[v])
        if case.get("mixed"):
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed)[v])
            if v in (0, 2):
                view["depth_z"] = torch.from_numpy(synthetic.synthetic_sparse_depth(n, h, w, seed)[v])
            if v in (0, 1):
                view["camera_poses"] = torch.from_numpy(synthetic.synthetic_poses(n, seed)[v])
            view["is_metric_scale"] = torch.tensor([v != 2])
        views.append(view)
    return views

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
    "cfg2_518": dict(views=8, h=518, w=518, seed=2),   # configs[1] at its real size (the bench's input seed)
    # configs[3] at its real size: 32 views + intrinsics + 90 %-sparse depth + metric flag
    "cfg4_518": dict(views=32, h=518, w=518, seed=4, multimodal=True),
    # two scenes per view (batch_size_per_view = 2, reference model.py:687), mixed geometric inputs
    "b2_224": dict(views=3, h=224, w=224, seed=12, mixed=True, batch=2),
}


# Info-sharing variants (make_golden.py VARIANTS): the reference rebuilt with these info_sharing_configs
VARIANT_CASES = ("gat_224", "aatpe_224", "aatnoref_224", "aat48_224")


def variant_config(name):
    """(full model config, case) of a variant fixture: the released config with the info_sharing_config the
    reference was built with (recorded in golden_meta.json)."""
    meta = json.load(open(os.path.join(HERE, "golden", "golden_meta.json")))[name]
    cfg = released_config()
    cfg["info_sharing_config"] = meta["info_sharing_config"]
    case = {k: meta[k] for k in ("views", "h", "w", "seed")}
    return cfg, case


def make_views(case):
    """Seeded reference-format views: images (+ intrinsics / sparse depth_z / 4x4 poses / is_metric_scale)."""
    import torch

    from mapanything.utils import synthetic

    n, h, w, seed = case["views"], case["h"], case["w"], case["seed"]
    B = case.get("batch", 1)  # scenes per view (batch_size_per_view, reference model.py:687)
    imgs = synthetic.synthetic_images(n, h, w, seed, batch=B)
    views = []
    for v in range(n):
        view = {"img": torch.from_numpy(imgs[v]), "data_norm_type": ["dinov2"]}
        if case.get("multimodal"):
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed, batch=B)[v])
            view["depth_z"] = torch.from_numpy(synthetic.synthetic_sparse_depth(n, h, w, seed, batch=B)[v])
            view["is_metric_scale"] = torch.ones(B, dtype=torch.bool)
        if case.get("rays_only"):
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed, batch=B)[v])
        if case.get("mixed"):
            # 3 views: intrinsics everywhere, depth on views 0 and 2, poses on views 0 and 1; scene 0: view 2 not
            # metric, further scenes: only view 0 metric
            view["intrinsics"] = torch.from_numpy(synthetic.synthetic_intrinsics(n, h, w, seed, batch=B)[v])
            if v in (0, 2):
                view["depth_z"] = torch.from_numpy(synthetic.synthetic_sparse_depth(n, h, w, seed, batch=B)[v])
            if v in (0, 1):
                view["camera_poses"] = torch.from_numpy(synthetic.synthetic_poses(n, seed, batch=B)[v])
            view["is_metric_scale"] = torch.tensor([(v != 2) if b == 0 else (v == 0) for b in range(B)])
        views.append(view)
    return views


IMAGE_FILES = [("a_land.jpg", 700, 520), ("b_land.png", 640, 480), ("c_small.png", 160, 120),
               ("d_portrait.png", 300, 420), ("e_notes.txt", 0, 0), ("f_portrait.jpg", 240, 360)]


def synthetic_image(W, H, seed):
    """Smooth seeded RGB image (gradients + discs + mild noise) as a uint8 (H, W, 3) array."""
    import numpy as np

    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.stack([x / max(W - 1, 1), y / max(H - 1, 1), (x + y) / max(W + H - 2, 1)], -1) * 200.0
    for _ in range(4):
        cx, cy, r = rng.uniform(0, W), rng.uniform(0, H), rng.uniform(0.1, 0.3) * min(W, H)
        img[(x - cx) ** 2 + (y - cy) ** 2 < r * r] += rng.uniform(-60, 60, 3)
    img += rng.normal(0, 3, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def write_image_files(folder):
    """The input files of the image-pipeline fixtures (PIL encodes them deterministically)."""
    import os

    import PIL.Image

    os.makedirs(folder, exist_ok=True)
    for i, (name, W, H) in enumerate(IMAGE_FILES):
        path = os.path.join(folder, name)
        if name.endswith(".txt"):
            open(path, "w").write("not an image\n")
        elif name.endswith(".jpg"):
            PIL.Image.fromarray(synthetic_image(W, H, 100 + i)).save(path, quality=90)
        else:
            PIL.Image.fromarray(synthetic_image(W, H, 100 + i)).save(path)
    return [n for n, _, _ in IMAGE_FILES]

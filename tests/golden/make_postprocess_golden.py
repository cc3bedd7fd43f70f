"""Generate the post-processing mask fixtures from the REAL reference (build container only).

    python tests/golden/make_postprocess_golden.py      # writes tests/golden/golden_postprocess.npz

Runs the reference's own `postprocess_model_outputs_for_inference` (mapanything/utils/inference.py:314-506:
points_to_normals geometry.py:1788-1851, normals_edge :2200-2259, depth_edge :2102-2143, max_pool_2d NaN
padding :1976-2090, torch.quantile confidence threshold, rgb() image.py:93-131) on the seeded scenes of
postprocess_cases.py for every option set, and stores data only: the final boolean masks (bit-packed), the
masked pts3d of the small case, img_no_norm and the recovered intrinsics.
"""

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import postprocess_cases as pc  # noqa: E402
import ref_harness  # noqa: E402


def main():
    ref_harness.install_stubs()
    if ref_harness.REF not in sys.path:
        sys.path.insert(0, ref_harness.REF)
    from mapanything.utils.inference import postprocess_model_outputs_for_inference  # noqa: E402

    out = {}
    for name, case in pc.CASES.items():
        sc = pc.make_scene(case)
        V, H, W = case["views"], case["h"], case["w"]
        for oi, opt in enumerate(pc.OPTIONS):
            raw, views = [], []
            for v in range(V):
                raw.append({
                    "pts3d": torch.from_numpy(sc["pts3d"][v:v + 1].copy()),
                    "pts3d_cam": torch.from_numpy(sc["pts3d_cam"][v:v + 1].copy()),
                    "ray_directions": torch.from_numpy(sc["ray_directions"][v:v + 1].copy()),
                    "depth_along_ray": torch.from_numpy(sc["depth_along_ray"][v:v + 1].copy()),
                    "conf": torch.from_numpy(sc["conf"][v:v + 1].copy()),
                    "non_ambiguous_mask": torch.from_numpy(sc["non_ambiguous_mask"][v:v + 1].copy()),
                    "cam_trans": torch.from_numpy(sc["cam_trans"][v:v + 1].copy()),
                    "cam_quats": torch.from_numpy(sc["cam_quats"][v:v + 1].copy()),
                })
                views.append({"img": torch.from_numpy(sc["img"][v:v + 1].copy()), "data_norm_type": ["dinov2"]})
            t0 = time.time()
            res = postprocess_model_outputs_for_inference(raw, views, apply_mask=True, **opt)
            dt = time.time() - t0
            mask = np.stack([r["mask"][0, ..., 0].numpy() for r in res], 0)
            out[f"{name}_{pc.option_key(oi)}_mask"] = np.packbits(mask.reshape(-1))
            if name == "pp_small":
                out[f"{name}_{pc.option_key(oi)}_pts3d"] = np.stack([r["pts3d"][0].numpy() for r in res], 0)
                out[f"{name}_{pc.option_key(oi)}_depth_along_ray"] = np.stack(
                    [r["depth_along_ray"][0].numpy() for r in res], 0)
            if oi == 0:
                out[f"{name}_intrinsics"] = np.stack([r["intrinsics"][0].numpy() for r in res], 0)
            if oi == 0 and name != "pp_518":  # img_no_norm of random pixels does not compress: small cases only
                out[f"{name}_img_no_norm"] = np.stack([np.asarray(r["img_no_norm"])[0] for r in res], 0).astype(
                    np.float32)
            print(name, oi, f"{dt:.2f}s", "kept", int(mask.sum()), "of", mask.size)
    np.savez_compressed(os.path.join(HERE, "golden_postprocess.npz"), **out)
    print("done")


if __name__ == "__main__":
    main()

"""Fixtures of the input pipeline (image.py:134-690, cropping.py:188-465) from the REAL reference, run here only.

    python tests/golden/make_image_golden.py      # writes tests/golden/golden_images.npz

The reference's image.py is imported through ref_harness (stubbed non-arithmetic imports).  Two of its
dependencies are absent from this image and are stood in for as follows:
  * torchvision.transforms ToTensor / Normalize / Compose: restated exactly as torchvision implements them for an
    RGB PIL image (uint8 HWC -> CHW float32 / 255; (x - mean) / std in float32);
  * cv2: only its nearest-neighbour resize of depth maps is used by these functions; no fixture case passes a
    depth map, so that path is not pinned here (tests/test_image_pipeline.py holds known answers for it).
Inputs are the seeded files of tests_helpers.write_image_files (regenerated identically by the tests).
Saved per case: the resized + cropped uint8 image (before normalisation) and the normalised image (both strided
[::7, ::7] for the 512/518-wide cases), true_shape and, for preprocess_inputs, intrinsics / poses.
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import ref_harness  # noqa: E402
from tests_helpers import synthetic_image, write_image_files  # noqa: E402

STRIDE = 7  # normalised 518-wide images are stored at [::7, ::7]


class ToTensor:
    def __call__(self, pic):
        a = np.array(pic, np.uint8, copy=True)
        return torch.from_numpy(a).permute(2, 0, 1).contiguous().to(torch.float32).div(255)


class Normalize:
    def __init__(self, mean, std):
        self.mean = torch.as_tensor(mean, dtype=torch.float32)
        self.std = torch.as_tensor(std, dtype=torch.float32)

    def __call__(self, t):
        return t.sub(self.mean[:, None, None]).div(self.std[:, None, None])


class Compose:
    def __init__(self, fs):
        self.fs = fs

    def __call__(self, x):
        for f in self.fs:
            x = f(x)
        return x


def main():
    ref_harness.install_stubs()
    tvt = sys.modules["torchvision.transforms"]
    tvt.ToTensor, tvt.Normalize, tvt.Compose = ToTensor, Normalize, Compose

    def no_cv2(*a, **k):
        raise NotImplementedError("cv2 path not pinned")

    sys.modules["cv2"].resize = no_cv2
    if ref_harness.REF not in sys.path:
        sys.path.insert(0, ref_harness.REF)
    from mapanything.utils import cropping as rc  # noqa: E402
    from mapanything.utils import image as ri  # noqa: E402

    out = {}
    with tempfile.TemporaryDirectory() as d:
        names = write_image_files(d)
        cases = {"fixed": dict(folder_or_list=d),
                 "square_s2": dict(folder_or_list=[os.path.join(d, n) for n in names], resize_mode="square",
                                   size=224, stride=2),
                 "long_portrait": dict(folder_or_list=[os.path.join(d, n) for n in names if "portrait" in n],
                                       resize_mode="longest_side", size=280),
                 "fixed_size": dict(folder_or_list=d, resize_mode="fixed_size", size=(230, 170)),
                 "fixed512": dict(folder_or_list=[os.path.join(d, n) for n in names[:2]], resolution_set=512,
                                  norm_type="dust3r")}
        for cname, kw in cases.items():
            res = ri.load_images(**kw)
            imgs = torch.cat([r["img"] for r in res], 0).numpy()
            step = STRIDE if imgs.shape[-1] > 300 else 1
            out[f"{cname}__norm"] = imgs[:, :, ::step, ::step]
            out[f"{cname}__true_shape"] = np.concatenate([r["true_shape"] for r in res], 0)
            # the uint8 image each view was normalised from (reference crop_resize_if_necessary on the same file)
            W, H = res[0]["true_shape"][0][::-1]
            files = kw["folder_or_list"]
            files = [os.path.join(d, n) for n in sorted(os.listdir(d))] if isinstance(files, str) else files
            keep = [f for i, f in enumerate(files) if i % kw.get("stride", 1) == 0
                    and f.lower().endswith((".jpg", ".jpeg", ".png"))]
            import PIL.Image
            from PIL.ImageOps import exif_transpose
            u8 = [np.asarray(rc.crop_resize_if_necessary(exif_transpose(PIL.Image.open(f)).convert("RGB"),
                                                         resolution=(int(W), int(H)))[0]) for f in keep]
            out[f"{cname}__u8"] = np.stack(u8, 0)[:, ::step, ::step]
            out[f"{cname}__step"] = np.int32(step)
    # preprocess_inputs: numpy / float tensor / PIL images, intrinsics and poses, no depth
    import PIL.Image
    K0 = np.array([[420.0, 0, 205.3], [0, 415.0, 148.9], [0, 0, 1]], np.float32)
    K1 = np.array([[300.0, 0, 160.0], [0, 300.0, 120.0], [0, 0, 1]], np.float32)
    pose = np.eye(4, dtype=np.float32)
    pose[:3, 3] = (0.3, -0.2, 1.5)
    views = [dict(img=synthetic_image(410, 300, 7), intrinsics=K0, camera_poses=pose, is_metric_scale=True),
             dict(img=torch.from_numpy(synthetic_image(320, 240, 8)).float() / 255.0, intrinsics=torch.from_numpy(K1),
                  camera_poses=(np.array([0, 0, 0, 1], np.float32), np.array([1, 2, 3], np.float32))),
             dict(img=PIL.Image.fromarray(synthetic_image(400, 310, 9)), instance="x")]
    pv = ri.preprocess_inputs(views, resize_mode="fixed_size", size=(224, 168))
    out["pre__norm"] = torch.cat([v["img"] for v in pv], 0).numpy()
    out["pre__K0"] = pv[0]["intrinsics"].numpy()
    out["pre__K1"] = pv[1]["intrinsics"].numpy()
    out["pre__pose0"] = pv[0]["camera_poses"].numpy()
    out["pre__q1"] = pv[1]["camera_poses"][0].numpy()
    out["pre__t1"] = pv[1]["camera_poses"][1].numpy()
    out["pre__keys"] = np.array([",".join(v.keys()) for v in pv])
    np.savez_compressed(os.path.join(HERE, "golden_images.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()

"""Input pipeline (mapanything/utils/image.py, cropping.py) against fixtures made by the reference's own
load_images / preprocess_inputs (tests/golden/make_image_golden.py).  Host parts (decode, target size, Lanczos /
bicubic resize, crop, intrinsics) are checked on the CPU; the GPU normalisation kernel bit-exactly on the GPU."""

import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from tests_helpers import synthetic_image, write_image_files

CASES = {"fixed": dict(), "square_s2": dict(resize_mode="square", size=224, stride=2),
         "long_portrait": dict(resize_mode="longest_side", size=280),
         "fixed_size": dict(resize_mode="fixed_size", size=(230, 170)),
         "fixed512": dict(resolution_set=512, norm_type="dust3r")}


@pytest.fixture(scope="module")
def fx():
    with np.load(os.path.join(GOLDEN, "golden_images.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("imgs"))
    names = write_image_files(d)
    return d, names


def _source(case, d, names):
    if case == "fixed" or case == "fixed_size":
        return d
    if case == "square_s2":
        return [os.path.join(d, n) for n in names]
    if case == "long_portrait":
        return [os.path.join(d, n) for n in names if "portrait" in n]
    return [os.path.join(d, n) for n in names[:2]]


def _preprocess_views():
    import PIL.Image

    K0 = np.array([[420.0, 0, 205.3], [0, 415.0, 148.9], [0, 0, 1]], np.float32)
    K1 = np.array([[300.0, 0, 160.0], [0, 300.0, 120.0], [0, 0, 1]], np.float32)
    pose = np.eye(4, dtype=np.float32)
    pose[:3, 3] = (0.3, -0.2, 1.5)
    return [dict(img=synthetic_image(410, 300, 7), intrinsics=K0, camera_poses=pose, is_metric_scale=True),
            dict(img=torch.from_numpy(synthetic_image(320, 240, 8)).float() / 255.0, intrinsics=torch.from_numpy(K1),
                 camera_poses=(np.array([0, 0, 0, 1], np.float32), np.array([1, 2, 3], np.float32))),
            dict(img=PIL.Image.fromarray(synthetic_image(400, 310, 9)), instance="x")]


@pytest.mark.parametrize("case", list(CASES))
def test_host_resize_crop_matches_reference(fx, files, case):
    from mapanything.utils.image import load_resized_images

    d, names = files
    kw = {k: v for k, v in CASES[case].items() if k != "norm_type"}
    imgs = load_resized_images(_source(case, d, names), **kw)
    step = int(fx[f"{case}__step"])
    u8 = np.stack([np.asarray(i) for i in imgs], 0)[:, ::step, ::step]
    assert np.array_equal(u8, fx[f"{case}__u8"])
    assert np.array_equal(np.int32([i.size[::-1] for i in imgs]), fx[f"{case}__true_shape"])


def test_host_preprocess_inputs_matches_reference(fx):
    from mapanything.utils.image import preprocess_inputs_host

    imgs, views = preprocess_inputs_host(_preprocess_views(), resize_mode="fixed_size", size=(224, 168))
    assert all(i.size == (224, 168) for i in imgs)
    np.testing.assert_allclose(views[0]["intrinsics"].numpy(), fx["pre__K0"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(views[1]["intrinsics"].numpy(), fx["pre__K1"], rtol=0, atol=1e-5)
    assert np.array_equal(views[0]["camera_poses"].numpy(), fx["pre__pose0"])
    assert np.array_equal(views[1]["camera_poses"][0].numpy(), fx["pre__q1"])
    assert np.array_equal(views[1]["camera_poses"][1].numpy(), fx["pre__t1"])
    keys = [",".join(["img", "data_norm_type"] + list(v.keys())) for v in views]
    assert keys == list(fx["pre__keys"])


def test_target_size_rules():
    from mapanything.utils.image import find_closest_aspect_ratio, target_size_for

    assert find_closest_aspect_ratio(4 / 3, 518) == (518, 392)
    assert find_closest_aspect_ratio(0.7, 518) == (336, 518)
    assert find_closest_aspect_ratio(1.0, 512) == (512, 512)
    assert target_size_for([2.0], "longest_side", 518, 14, 518) == (518, 252)
    assert target_size_for([0.5], "longest_side", 518, 14, 518) == (252, 518)
    assert target_size_for([1.3], "square", 300, 14, 518) == (294, 294)
    assert target_size_for([1.3], "fixed_size", (230, 170), 14, 518) == (224, 168)


def test_nearest_resize_follows_opencv_rule():
    """cv2.INTER_NEAREST with an explicit dsize: src = min(floor(dst * (1 / (dsize / ssize))), ssize - 1).
    OpenCV is absent here: known answers of that rule (parity with cv2 itself unpinned)."""
    from mapanything.utils.cropping import _resize_nearest

    a = np.arange(12, dtype=np.float32).reshape(3, 4)
    assert np.array_equal(_resize_nearest(a, (2, 3)), a[:, [0, 2]])
    b = np.arange(3, dtype=np.float32)[None]
    assert np.array_equal(_resize_nearest(b, (5, 1))[0], np.float32([0, 0, 1, 1, 2]))
    c = np.arange(49, dtype=np.float32).reshape(7, 7)
    assert np.array_equal(_resize_nearest(c, (3, 3)), c[np.ix_([0, 2, 4], [0, 2, 4])])


def test_argument_errors_like_reference(files):
    from mapanything.utils.image import load_resized_images, preprocess_inputs_host

    d, _ = files
    with pytest.raises(ValueError, match="Resize_mode"):
        load_resized_images(d, resize_mode="bogus")
    with pytest.raises(ValueError, match="Size parameter"):
        load_resized_images(d, resize_mode="square")
    with pytest.raises(ValueError, match="Size must be a tuple"):
        load_resized_images(d, resize_mode="fixed_size", size=224)
    with pytest.raises(ValueError, match="Unknown image normalization"):
        load_resized_images(d, norm_type="nope")
    with pytest.raises(ValueError, match="No valid images"):
        load_resized_images([os.path.join(d, "e_notes.txt")])
    with pytest.raises(ValueError, match="cannot have both"):
        preprocess_inputs_host([dict(img=synthetic_image(32, 32, 1), intrinsics=np.eye(3, dtype=np.float32),
                                     ray_directions=np.zeros((32, 32, 3), np.float32))])
    with pytest.raises(ValueError, match="cannot be empty"):
        preprocess_inputs_host([])


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("gpu_resize", [True, False], ids=["gpu_resize", "pil_resize"])
@pytest.mark.parametrize("case", list(CASES))
def test_load_images_matches_reference(fx, files, case, gpu_resize):
    from mapanything.utils.image import load_images

    d, names = files
    res = load_images(_source(case, d, names), gpu_resize=gpu_resize, **CASES[case])
    step = int(fx[f"{case}__step"])
    imgs = torch.cat([r["img"] for r in res], 0)
    assert imgs.is_cuda and imgs.dtype == torch.float32
    assert np.array_equal(imgs.cpu().numpy()[:, :, ::step, ::step], fx[f"{case}__norm"])  # bit-exact
    assert np.array_equal(np.concatenate([r["true_shape"] for r in res], 0), fx[f"{case}__true_shape"])
    assert [r["idx"] for r in res] == list(range(len(res))) and res[0]["instance"] == "0"
    assert res[0]["data_norm_type"] == [CASES[case].get("norm_type", "dinov2")]


@pytest.mark.gpu
def test_iter_load_images_prefetch_matches_load_images(fx, files):
    """The prefetching scene iterator (host decode / resize of scene k+1 under the caller's work on scene k) yields
    exactly load_images' views for every scene, in order — the reference fixtures included."""
    from mapanything.utils.image import iter_load_images, load_images

    d, names = files
    scenes = [_source(c, d, names) for c in CASES]
    kws = [CASES[c] for c in CASES]
    # one keyword set per stream: the iterator takes the same arguments as load_images
    for prefetch, gr in ((1, True), (2, True), (1, False)):
        for sc, kw, c, got in zip(scenes, kws, CASES, (next(iter_load_images([s], prefetch=prefetch, gpu_resize=gr, **k))
                                                       for s, k in zip(scenes, kws))):
            ref = load_images(sc, gpu_resize=gr, **kw)
            assert len(got) == len(ref)
            for a, b in zip(got, ref):
                assert torch.equal(a["img"], b["img"]) and np.array_equal(a["true_shape"], b["true_shape"])
    seq = list(iter_load_images([scenes[0]] * 3, prefetch=2))
    step = int(fx["fixed__step"])
    for views in seq:
        imgs = torch.cat([r["img"] for r in views], 0)
        assert np.array_equal(imgs.cpu().numpy()[:, :, ::step, ::step], fx["fixed__norm"])


@pytest.mark.gpu
def test_preprocess_inputs_matches_reference(fx):
    from mapanything.utils.image import preprocess_inputs

    views = preprocess_inputs(_preprocess_views(), resize_mode="fixed_size", size=(224, 168))
    assert np.array_equal(torch.cat([v["img"] for v in views], 0).cpu().numpy(), fx["pre__norm"])
    assert [",".join(v.keys()) for v in views] == list(fx["pre__keys"])


@pytest.mark.gpu
def test_preprocess_inputs_ray_directions_recover_intrinsics():
    """A view given as ray directions is turned into intrinsics (geometry.py:304-447) before resizing."""
    from mapanything.utils.image import preprocess_inputs

    K = np.array([[250.0, 0, 159.5], [0, 260.0, 119.5], [0, 0, 1]], np.float32)
    H, W = 240, 320
    y, x = np.mgrid[0:H, 0:W].astype(np.float32)
    rays = np.stack([(x - K[0, 2]) / K[0, 0], (y - K[1, 2]) / K[1, 1], np.ones_like(x)], -1)
    rays /= np.linalg.norm(rays, axis=-1, keepdims=True)
    a = preprocess_inputs([dict(img=synthetic_image(W, H, 3), ray_directions=rays)], resize_mode="fixed_size",
                          size=(224, 168))
    b = preprocess_inputs([dict(img=synthetic_image(W, H, 3), intrinsics=K)], resize_mode="fixed_size",
                          size=(224, 168))
    np.testing.assert_allclose(a[0]["intrinsics"].numpy(), b[0]["intrinsics"].numpy(), rtol=1e-4, atol=1e-3)
    assert torch.equal(a[0]["img"], b[0]["img"])


@pytest.mark.parametrize("case", list(CASES))
def test_gpu_resize_host_stage_matches_pil(files, case):
    """Host stage of the GPU-resize loader (decode + resize_geometry + the fixed-point plans), run through the
    kernels' integer arithmetic in numpy (test_resample_plan.passes), equals the PIL path image for image."""
    from mapanything.utils.image import _decode_scene_for_gpu, load_resized_images
    from test_resample_plan import passes

    d, names = files
    kw = {k: v for k, v in CASES[case].items()}
    ref = load_resized_images(_source(case, d, names), **kw)
    scene = _decode_scene_for_gpu(_source(case, d, names), **kw)
    assert len(scene.images) == len(ref)
    for (src, blob), im in zip(scene.images, ref):
        got = passes(src.numpy(), blob)
        assert tuple(scene.target) == im.size and np.array_equal(got, np.asarray(im))

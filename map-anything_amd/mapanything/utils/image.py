"""Input pipeline: load / resize / crop / normalise images (+ their depth maps and intrinsics) into the views
`MapAnything.infer` takes (reference: mapanything/utils/image.py:37-690).

Decoding, resampling and cropping run on the host with PIL exactly as in the reference (same library, same
Lanczos / bicubic filters, same crop boxes); the uint8 images then go to the GPU in one copy (4x fewer bytes than
the float tensors) and ToTensor + Normalize runs there (`mapa_normalize_image`, bit-identical to torchvision's two
float32 operations).  The returned views hold device tensors, ready for infer() without another H2D copy.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from typing import List

import numpy as np
import PIL.Image
import torch
from PIL.ImageOps import exif_transpose

from .. import _native as nat
from .cropping import crop_resize_if_necessary

# uniception/models/encoders/image_normalizations.py:17-35 (float32 like the reference's torch tensors)
IMAGE_NORMALIZATION_DICT = {
    "dummy": ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    "croco": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
    "dust3r": ((0.5, 0.5, 0.5), (0.5, 0.5, 0.5)),
    "dinov2": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
    "identity": ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    "patch_embedder": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
    "radio": ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    "sea_raft": ((0.0, 0.0, 0.0), tuple(np.float32(np.float32(1.0) / np.float32(255.0)) for _ in range(3))),
    "unimatch": ((0.0, 0.0, 0.0), tuple(np.float32(np.float32(1.0) / np.float32(255.0)) for _ in range(3))),
    "roma": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
    "cosmos": ((0.0, 0.0, 0.0), (0.5, 0.5, 0.5)),
}

# image.py:37-69: fixed (width, height) per aspect ratio, multiples of the patch size
RESOLUTION_MAPPINGS = {
    518: {1.000: (518, 518), 1.321: (518, 392), 1.542: (518, 336), 1.762: (518, 294), 2.056: (518, 252),
          3.083: (518, 168), 0.757: (392, 518), 0.649: (336, 518), 0.567: (294, 518), 0.486: (252, 518)},
    512: {1.000: (512, 512), 1.333: (512, 384), 1.524: (512, 336), 1.778: (512, 288), 2.000: (512, 256),
          3.200: (512, 160), 0.750: (384, 512), 0.656: (336, 512), 0.562: (288, 512), 0.500: (256, 512)},
}
ASPECT_RATIO_KEYS = {k: sorted(v.keys()) for k, v in RESOLUTION_MAPPINGS.items()}
RESIZE_MODES = ("fixed_mapping", "longest_side", "square", "fixed_size")
IMAGE_EXTENSIONS = (".jpg", ".jpeg", ".png")


def find_closest_aspect_ratio(aspect_ratio, resolution_set):
    """image.py:71-86: the mapping entry whose aspect-ratio key is closest (first one on ties)."""
    keys = ASPECT_RATIO_KEYS[resolution_set]
    return RESOLUTION_MAPPINGS[resolution_set][min(keys, key=lambda x: abs(x - aspect_ratio))]


def _check_resize_args(resize_mode, size):
    """image.py:164-190 / 370-396."""
    if resize_mode not in RESIZE_MODES:
        raise ValueError(f"Resize_mode must be one of {list(RESIZE_MODES)}, got '{resize_mode}'")
    if resize_mode in ("longest_side", "square", "fixed_size") and size is None:
        raise ValueError(f"Size parameter is required for resize_mode='{resize_mode}'")
    if resize_mode in ("longest_side", "square"):
        if not isinstance(size, int):
            raise ValueError(f"Size must be an int for resize_mode='{resize_mode}', got {type(size)}")
    elif resize_mode == "fixed_size":
        if not isinstance(size, (tuple, list)) or len(size) != 2:
            raise ValueError(f"Size must be a tuple/list of (width, height) for resize_mode='fixed_size', got {size}")
        if not all(isinstance(x, int) for x in size):
            raise ValueError(f"Size values must be integers for resize_mode='fixed_size', got {size}")


def target_size_for(aspect_ratios: List[float], resize_mode, size, patch_size, resolution_set):
    """image.py:238-275: one (width, height) for every view, from the mean aspect ratio."""
    avg = sum(aspect_ratios) / len(aspect_ratios)
    if resize_mode == "fixed_mapping":
        return tuple(find_closest_aspect_ratio(avg, resolution_set))
    if resize_mode == "square":
        s = round(size // patch_size) * patch_size
        return (s, s)
    if resize_mode == "longest_side":
        if avg >= 1:
            return (size, round((size // patch_size) / avg) * patch_size)
        return (round((size // patch_size) * avg) * patch_size, size)
    return ((size[0] // patch_size) * patch_size, (size[1] // patch_size) * patch_size)


def _norm_consts(norm_type):
    if norm_type not in IMAGE_NORMALIZATION_DICT:
        raise ValueError(f"Unknown image normalization type: {norm_type}. Available options: "
                         f"{list(IMAGE_NORMALIZATION_DICT.keys())}")
    return IMAGE_NORMALIZATION_DICT[norm_type]


def normalize_images(pil_images: List[PIL.Image.Image], norm_type="dinov2", device=None) -> torch.Tensor:
    """ToTensor + Normalize of same-size RGB images on the GPU -> (n, 3, H, W) float32 on `device`."""
    mean, std = _norm_consts(norm_type)
    arr = np.stack([np.asarray(im, dtype=np.uint8) for im in pil_images], 0)  # (n, H, W, 3)
    n, H, W, _ = arr.shape
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    u8 = torch.from_numpy(arr).pin_memory().to(dev, non_blocking=True)
    out = torch.empty(n, 3, H, W, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        nat.normalize_image(u8, n, H, W, mean, std, out)
    return out


def _decode_scene(folder_or_list, resize_mode, size, norm_type, patch_size, verbose, bayer_format, resolution_set,
                  stride, pool):
    """image.py:163-275: decode every image (EXIF-transposed RGB; unreadable files skipped) and choose the common
    target size.  Returns (decoded PIL images, (width, height))."""
    _check_resize_args(resize_mode, size)
    if bayer_format:
        raise NotImplementedError("bayer_format needs OpenCV's demosaicing, which this image does not ship")
    if isinstance(folder_or_list, str):
        root, content = folder_or_list, sorted(os.listdir(folder_or_list))
    elif isinstance(folder_or_list, list):
        root, content = "", folder_or_list
    else:
        raise ValueError(f"Bad {folder_or_list=} ({type(folder_or_list)})")
    _norm_consts(norm_type)
    paths = [p for i, p in enumerate(content) if i % stride == 0 and p.lower().endswith(IMAGE_EXTENSIONS)]

    def decode(path):
        try:
            return exif_transpose(PIL.Image.open(os.path.join(root, path))).convert("RGB")
        except Exception as e:  # unreadable files are skipped, as in the reference
            if verbose:
                print(f"Warning: Could not load {path}: {e}")
            return None

    loaded = [im for im in pool.map(decode, paths) if im is not None]
    if not loaded:
        raise ValueError("No valid images found")
    target = target_size_for([im.size[0] / im.size[1] for im in loaded], resize_mode, size, patch_size,
                             resolution_set)
    if verbose:
        print(f"Using target resolution {target[0]}x{target[1]} (W x H) for all images")
    return loaded, target


def load_resized_images(folder_or_list, resize_mode="fixed_mapping", size=None, norm_type="dinov2", patch_size=14,
                        verbose=False, bayer_format=False, resolution_set=518, stride=1, num_workers=None):
    """Host part of load_images (image.py:163-303) on PIL: decode, choose the common target size, Lanczos / bicubic
    resize + crop.  Returns the resized PIL images (the host reference of the GPU resize)."""
    n_hint = len(folder_or_list) if isinstance(folder_or_list, list) else None
    # PIL decodes and resamples with the GIL released: a thread pool keeps every host core busy (file order kept)
    with ThreadPoolExecutor(max_workers=_workers(num_workers, n_hint)) as pool:
        loaded, target = _decode_scene(folder_or_list, resize_mode, size, norm_type, patch_size, verbose,
                                       bayer_format, resolution_set, stride, pool)
        return list(pool.map(lambda im: crop_resize_if_necessary(im, resolution=target)[0], loaded))


def resize_geometry(in_wh, target_wh):
    """rescale_image_and_other_optional_info + the centred crop of crop_resize_if_necessary without intrinsics
    (cropping.py:188-280 / 385-465, numpy float64 like the reference): (resized (w, h), PIL filter, crop (left, top))."""
    input_resolution = np.array(in_wh)
    output_resolution = np.array(target_wh)
    scale_final = max(output_resolution / input_resolution) + 1e-8
    rs = np.floor(input_resolution * scale_final).astype(int)
    filt = nat.RESAMPLE_LANCZOS if scale_final < 1 else nat.RESAMPLE_BICUBIC
    w, h = int(rs[0]), int(rs[1])
    return (w, h), filt, ((w - int(target_wh[0])) // 2, (h - int(target_wh[1])) // 2)


class _DecodedScene:
    """Host stage of the GPU-resize loader: decoded uint8 images in pinned memory + their fixed-point resize plans
    (one pinned int32 blob), ready for one H2D copy each and the resize kernels."""

    def __init__(self, images, target, plans, offsets):
        self.images, self.target, self.plans, self.offsets = images, target, plans, offsets


def _decode_scene_for_gpu(folder_or_list, resize_mode="fixed_mapping", size=None, norm_type="dinov2", patch_size=14,
                          verbose=False, bayer_format=False, resolution_set=518, stride=1, num_workers=None):
    n_hint = len(folder_or_list) if isinstance(folder_or_list, list) else None
    with ThreadPoolExecutor(max_workers=_workers(num_workers, n_hint)) as pool:
        loaded, target = _decode_scene(folder_or_list, resize_mode, size, norm_type, patch_size, verbose,
                                       bayer_format, resolution_set, stride, pool)
        pin = torch.cuda.is_available()  # (the host stage alone also runs on a CPU-only machine: tests)

        def host_copy(im):  # the RGB bytes into pinned host memory, on the pool's threads
            t = torch.empty((im.size[1], im.size[0], 3), dtype=torch.uint8, pin_memory=pin)
            np.copyto(t.numpy(), np.asarray(im, dtype=np.uint8))
            return t
        pinned = list(pool.map(host_copy, loaded))
    blobs, offsets, off = [], [], 0
    for im in loaded:
        (rw, rh), filt, (left, top) = resize_geometry(im.size, target)
        b = nat.resize_plan(im.size[0], im.size[1], rw, rh, left, top, int(target[0]), int(target[1]), filt)
        blobs.append(b)
        offsets.append(off)
        off += (b.size + 63) // 64 * 64  # 256-B aligned plans
    plans = torch.zeros(off, dtype=torch.int32, pin_memory=pin)
    pn = plans.numpy()
    for b, o in zip(blobs, offsets):
        pn[o:o + b.size] = b
    return _DecodedScene(list(zip(pinned, blobs)), target, plans, offsets)


def _resize_on_gpu(scene: _DecodedScene, norm_type, device):
    """Device stage: H2D of the pinned images + plans (stream-ordered), PIL-exact resize + crop + normalise
    (mapa_resize_normalize) into one (n, 3, H, W) float32 batch."""
    mean, std = _norm_consts(norm_type)
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    tw, th = int(scene.target[0]), int(scene.target[1])
    with torch.cuda.device(dev):
        plans = scene.plans.to(dev, non_blocking=True)
        ws_bytes = max(nat.resize_workspace_bytes(b) for _, b in scene.images)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        out = torch.empty(len(scene.images), 3, th, tw, dtype=torch.float32, device=dev)
        for i, ((src, blob), off) in enumerate(zip(scene.images, scene.offsets)):
            d = src.to(dev, non_blocking=True)
            nat.resize_normalize(d, d.shape[1] * 3, blob, plans[off:], mean, std, out=out[i], workspace=ws)
    return out


def _views(imgs, shapes, norm_type):
    return [dict(img=imgs[i:i + 1], true_shape=np.int32([shapes[i]]), idx=i, instance=str(i),
                 data_norm_type=[norm_type]) for i in range(imgs.shape[0])]


def _workers(num_workers, n):
    if num_workers is None:
        num_workers = min(16, os.cpu_count() or 1)
    return max(1, min(int(num_workers), max(n or num_workers, 1)))


def _host_stage(folder_or_list, gpu_resize, **kw):
    if gpu_resize:
        return _decode_scene_for_gpu(folder_or_list, **kw)
    return load_resized_images(folder_or_list, **kw)


def _device_stage(host, norm_type, device):
    if isinstance(host, _DecodedScene):
        imgs = _resize_on_gpu(host, norm_type, device)
        return _views(imgs, [(int(host.target[1]), int(host.target[0]))] * imgs.shape[0], norm_type)
    imgs = normalize_images(host, norm_type, device)
    return _views(imgs, [im.size[::-1] for im in host], norm_type)


def load_images(folder_or_list, resize_mode="fixed_mapping", size=None, norm_type="dinov2", patch_size=14,
                verbose=False, bayer_format=False, resolution_set=518, stride=1, device=None, num_workers=None,
                gpu_resize=True):
    """image.py:134-333: open every image of a folder (sorted) or list, resize + crop all to one target size from
    their mean aspect ratio, normalise.  Returns [{img (1,3,H,W), true_shape, idx, instance, data_norm_type}] with
    img on `device` (default: the current GPU).

    gpu_resize=True (default): the host only decodes (PIL, thread pool); the Lanczos / bicubic resize, the crop and
    ToTensor + Normalize run on the GPU (mapa_resize_normalize, bit-identical with PIL's Image.resize).
    gpu_resize=False: PIL resizes on the host (load_resized_images), the GPU only normalises."""
    kw = dict(resize_mode=resize_mode, size=size, norm_type=norm_type, patch_size=patch_size, verbose=verbose,
              bayer_format=bayer_format, resolution_set=resolution_set, stride=stride, num_workers=num_workers)
    return _device_stage(_host_stage(folder_or_list, gpu_resize, **kw), norm_type, device)


def iter_load_images(scenes, prefetch=1, **kwargs):
    """Yield load_images(scene, **kwargs) for every scene (a folder or a file list) in order, with the host part of
    the next `prefetch` scenes (decode, plus the PIL resize when gpu_resize=False; PIL on host threads, GIL
    released) running while the caller works on the current one — so a stream of scenes fed to MapAnything.infer
    keeps the GPU busy instead of alternating host decode and GPU inference.  Each scene's images go to the GPU and
    are resized / normalised when the scene is yielded (stream-ordered behind the previous scene's work).  Results
    are exactly load_images' (the same functions, only overlapped)."""
    from concurrent.futures import ThreadPoolExecutor as _TPE

    scenes = list(scenes)
    device = kwargs.pop("device", None)
    gpu_resize = kwargs.pop("gpu_resize", True)
    norm_type = kwargs.get("norm_type", "dinov2")
    prefetch = max(1, int(prefetch))
    with _TPE(max_workers=prefetch) as ahead:
        pending = [ahead.submit(_host_stage, sc, gpu_resize, **kwargs) for sc in scenes[:prefetch]]
        for k in range(len(scenes)):
            host = pending.pop(0).result()
            if k + prefetch < len(scenes):
                pending.append(ahead.submit(_host_stage, scenes[k + prefetch], gpu_resize, **kwargs))
            yield _device_stage(host, norm_type, device)


def _to_pil(img, view_idx):
    """image.py:468-497."""
    if isinstance(img, torch.Tensor):
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError(f"Expected tensor shape (H, W, 3) for img in view {view_idx}, got {img.shape}")
        img = ((img * 255) if img.max() <= 1.0 else img).clamp(0, 255).byte().cpu().numpy()
        return PIL.Image.fromarray(img)
    if isinstance(img, np.ndarray):
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError(f"Expected array shape (H, W, 3) for img in view {view_idx}, got {img.shape}")
        if img.dtype != np.uint8:
            img = (img * 255).clip(0, 255).astype(np.uint8)
        return PIL.Image.fromarray(img)
    if isinstance(img, PIL.Image.Image):
        return img
    raise ValueError(f"Unsupported image type in view {view_idx}: {type(img)}")


def _to_numpy(data, expected_shape, name, view_idx):
    if isinstance(data, torch.Tensor):
        data = data.cpu().numpy()
    if not isinstance(data, np.ndarray):
        raise ValueError(f"Expected tensor or array for {name} in view {view_idx}, got {type(data)}")
    if expected_shape is not None and data.shape != expected_shape:
        raise ValueError(f"Expected shape {expected_shape} for {name} in view {view_idx}, got {data.shape}")
    return data


def _image_hw(img, view_idx):
    if isinstance(img, (torch.Tensor, np.ndarray)):
        if img.ndim == 3 and img.shape[2] == 3:
            return img.shape[0], img.shape[1]
        kind = "tensor" if isinstance(img, torch.Tensor) else "array"
        raise ValueError(f"Expected {kind} shape (H, W, 3) for img in view {view_idx}, got {img.shape}")
    if isinstance(img, PIL.Image.Image):
        return img.size[1], img.size[0]
    raise ValueError(f"Unsupported image type in view {view_idx}: {type(img)}")


def preprocess_inputs(input_views, resize_mode="fixed_mapping", size=None, norm_type="dinov2", patch_size=14,
                      resolution_set=518, verbose=False, device=None):
    """image.py:335-690: resize + crop every view's image, depth_z and intrinsics (ray_directions are turned into
    intrinsics first, on the GPU) to one target size, normalise the images (GPU), add the batch dimension to every
    input."""
    images, processed = preprocess_inputs_host(input_views, resize_mode, size, norm_type, patch_size,
                                               resolution_set, device)
    imgs = normalize_images(images, norm_type, device)
    return [{"img": imgs[i:i + 1], "data_norm_type": [norm_type], **p} for i, p in enumerate(processed)]


def preprocess_inputs_host(input_views, resize_mode="fixed_mapping", size=None, norm_type="dinov2", patch_size=14,
                           resolution_set=518, device=None):
    """Host part of preprocess_inputs: (resized PIL images, per-view dicts without img / data_norm_type)."""
    _check_resize_args(resize_mode, size)
    if not input_views:
        raise ValueError("input_views cannot be empty")
    ratios = []
    for i, view in enumerate(input_views):
        if "img" in view:
            H, W = _image_hw(view["img"], i)
            ratios.append(W / H)
    if not ratios:
        raise ValueError("No valid images found in input_views")
    target = target_size_for(ratios, resize_mode, size, patch_size, resolution_set)
    _norm_consts(norm_type)
    processed, images = [], []
    for i, view in enumerate(input_views):
        if "img" not in view:
            raise ValueError(f"View {i} missing required 'img' key")
        img = _to_pil(view["img"], i)
        depthmap = intrinsics = None
        if "depth_z" in view:
            depthmap = _to_numpy(view["depth_z"], None, "depth_z", i)
            if depthmap.ndim != 2:
                raise ValueError(f"Expected shape (H, W) for depth_z in view {i}, got {depthmap.shape}")
        if "intrinsics" in view and "ray_directions" in view:
            raise ValueError(f"View {i} cannot have both 'intrinsics' and 'ray_directions'. Please provide only one "
                             "as they are redundant (ray_directions can be used to recover intrinsics).")
        if "intrinsics" in view:
            intrinsics = _to_numpy(view["intrinsics"], (3, 3), "intrinsics", i)
        if "ray_directions" in view:
            rays = _to_numpy(view["ray_directions"], None, "ray_directions", i)
            if rays.ndim != 3 or rays.shape[2] != 3:
                raise ValueError(f"Expected shape (H, W, 3) for ray_directions in view {i}, got {rays.shape}")
            intrinsics = _recover_intrinsics(rays, device)
        res = crop_resize_if_necessary(image=img, resolution=target, depthmap=depthmap, intrinsics=intrinsics)
        out, k = {}, 1
        images.append(res[0])
        if depthmap is not None:
            out["depth_z"] = torch.from_numpy(np.ascontiguousarray(res[k]))[None]
            k += 1
        if intrinsics is not None:
            out["intrinsics"] = torch.from_numpy(np.ascontiguousarray(res[k]))[None]
            k += 1
        if "camera_poses" in view:
            out["camera_poses"] = _batched_poses(view["camera_poses"])
        for key, value in view.items():
            if key not in ("img", "depth_z", "intrinsics", "ray_directions", "camera_poses"):
                out[key] = value
        processed.append(out)
    return images, processed


def _recover_intrinsics(rays: np.ndarray, device) -> np.ndarray:
    """recover_pinhole_intrinsics_from_ray_directions (geometry.py:304-447) on the GPU (mapa_recover_intrinsics)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    H, W, _ = rays.shape
    r = torch.from_numpy(np.ascontiguousarray(rays, np.float32)).to(dev)[None]
    K = torch.empty(1, 3, 3, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        nat.recover_intrinsics(r, 1, H, W, K)
    return K[0].cpu().numpy()


def _batched_poses(camera_poses):
    """image.py:624-655: (quats, trans) tuple or a 4x4 matrix, each given a batch dimension."""
    def t(x):
        if isinstance(x, torch.Tensor):
            return x[None]
        if isinstance(x, np.ndarray):
            return torch.from_numpy(x)[None]
        return torch.tensor(x)[None]

    if isinstance(camera_poses, tuple):
        return (t(camera_poses[0]), t(camera_poses[1]))
    if isinstance(camera_poses, (torch.Tensor, np.ndarray)):
        return t(camera_poses)
    raise ValueError(f"Unsupported camera_poses format: {type(camera_poses)}. Expected tuple (quats, trans) or "
                     "matrix (tensor/array).")


def rgb(ftensor, norm_type, true_shape=None):
    """image.py:89-131: normalised image(s) -> RGB in [0, 1] (numpy, host-side visualisation helper)."""
    if isinstance(ftensor, list):
        return [rgb(x, norm_type, true_shape=true_shape) for x in ftensor]
    if isinstance(ftensor, torch.Tensor):
        ftensor = ftensor.detach().cpu().numpy()
    if ftensor.ndim == 3 and ftensor.shape[0] == 3:
        ftensor = ftensor.transpose(1, 2, 0)
    elif ftensor.ndim == 4 and ftensor.shape[1] == 3:
        ftensor = ftensor.transpose(0, 2, 3, 1)
    if true_shape is not None:
        H, W = true_shape
        ftensor = ftensor[:H, :W]
    if ftensor.dtype == np.uint8:
        img = np.float32(ftensor) / 255
    else:
        if norm_type in IMAGE_NORMALIZATION_DICT:
            mean, std = (np.asarray(x, np.float32) for x in IMAGE_NORMALIZATION_DICT[norm_type])
        elif norm_type == "identity":
            mean, std = 0.0, 1.0
        else:
            raise ValueError(f"Unknown image normalization type: {norm_type}. Available types: identity or "
                             f"{IMAGE_NORMALIZATION_DICT.keys()}")
        img = ftensor * std + mean
    return img.clip(min=0, max=1)

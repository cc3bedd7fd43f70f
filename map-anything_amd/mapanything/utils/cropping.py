"""Resize + crop of an image and its per-pixel / camera data to a target resolution (reference:
mapanything/utils/cropping.py, itself from DUSt3R).  Host-side: PIL does the image resampling exactly as in the
reference (same library, same filters), numpy does the nearest-neighbour resize of depth maps (the reference calls
cv2.resize(..., INTER_NEAREST); OpenCV is not in this image, so its nearest rule is restated in `_resize_nearest`).
"""
from __future__ import annotations

import numpy as np
import PIL.Image

LANCZOS = PIL.Image.Resampling.LANCZOS
BICUBIC = PIL.Image.Resampling.BICUBIC


def opencv_to_colmap_intrinsics(K):
    """geometry.py:1580-1591: pixel-centre convention (0,0) -> (0.5,0.5)."""
    K = K.copy()
    K[0, 2] += 0.5
    K[1, 2] += 0.5
    return K


def colmap_to_opencv_intrinsics(K):
    """geometry.py:1566-1577."""
    K = K.copy()
    K[0, 2] -= 0.5
    K[1, 2] -= 0.5
    return K


def _resize_nearest(a: np.ndarray, out_wh) -> np.ndarray:
    """cv2.resize(a, (W, H), interpolation=INTER_NEAREST) with an explicit dsize (fx / fy are then ignored):
    inv_scale = dsize / ssize, ifx = 1 / inv_scale (double), source index min(floor(dst * ifx), src - 1)
    (OpenCV cv::resize -> resizeNN)."""
    H, W = a.shape[:2]
    ow, oh = int(out_wh[0]), int(out_wh[1])
    ifx, ify = 1.0 / (ow / W), 1.0 / (oh / H)
    sx = np.minimum(np.floor(np.arange(ow, dtype=np.float64) * ifx).astype(np.int64), W - 1)
    sy = np.minimum(np.floor(np.arange(oh, dtype=np.float64) * ify).astype(np.int64), H - 1)
    return a[sy[:, None], sx[None, :]]


def camera_matrix_of_crop(input_camera_matrix, input_resolution, output_resolution, scaling=1, offset_factor=0.5,
                          offset=None):
    """cropping.py:283-317."""
    margins = np.asarray(input_resolution) * scaling - output_resolution
    assert np.all(margins >= 0.0)
    if offset is None:
        offset = offset_factor * margins
    K = opencv_to_colmap_intrinsics(input_camera_matrix)
    K[:2, :] *= scaling
    K[:2, 2] -= offset
    return colmap_to_opencv_intrinsics(K)


def rescale_image_and_other_optional_info(image, output_resolution, depthmap=None, camera_intrinsics=None,
                                          force=True, additional_quantities_to_be_resized_with_nearest=None):
    """cropping.py:188-280: scale so the target fits (Lanczos when shrinking, bicubic when growing)."""
    if not isinstance(image, PIL.Image.Image):
        image = PIL.Image.fromarray(image)
    input_resolution = np.array(image.size)  # (W, H)
    output_resolution = np.array(output_resolution)
    if depthmap is not None:
        assert tuple(depthmap.shape[:2]) == image.size[::-1]
    extra = additional_quantities_to_be_resized_with_nearest
    assert output_resolution.shape == (2,)
    scale_final = max(output_resolution / image.size) + 1e-8
    if scale_final >= 1 and not force:
        return image, depthmap, camera_intrinsics, extra
    output_resolution = np.floor(input_resolution * scale_final).astype(int)
    image = image.resize(tuple(int(x) for x in output_resolution), resample=LANCZOS if scale_final < 1 else BICUBIC)
    if depthmap is not None:
        depthmap = _resize_nearest(depthmap, output_resolution)
    if extra is not None:
        extra = [_resize_nearest(q, output_resolution) for q in extra]
    if camera_intrinsics is not None:
        camera_intrinsics = camera_matrix_of_crop(camera_intrinsics, input_resolution, output_resolution,
                                                  scaling=scale_final)
    return image, depthmap, camera_intrinsics, extra


def crop_image_and_other_optional_info(image, crop_bbox, depthmap=None, camera_intrinsics=None,
                                       additional_quantities=None):
    """cropping.py:320-360."""
    left, top, right, bottom = (int(x) for x in crop_bbox)
    image = image.crop((left, top, right, bottom))
    if depthmap is not None:
        depthmap = depthmap[top:bottom, left:right]
    if additional_quantities is not None:
        additional_quantities = [q[top:bottom, left:right] for q in additional_quantities]
    if camera_intrinsics is not None:
        camera_intrinsics = camera_intrinsics.copy()
        camera_intrinsics[0, 2] -= left
        camera_intrinsics[1, 2] -= top
    return image, depthmap, camera_intrinsics, additional_quantities


def bbox_from_intrinsics_in_out(input_camera_matrix, output_camera_matrix, output_resolution):
    """cropping.py:363-382."""
    out_width, out_height = output_resolution
    left, top = np.int32(np.round(input_camera_matrix[:2, 2] - output_camera_matrix[:2, 2]))
    return (left, top, left + out_width, top + out_height)


def crop_resize_if_necessary(image, resolution, depthmap=None, intrinsics=None, additional_quantities=None):
    """cropping.py:385-465: rescale so the target fits, then crop (centred on the principal point when the
    intrinsics are known, on the image centre otherwise).  Returns (image[, depth][, intrinsics][, extra])."""
    if not isinstance(image, PIL.Image.Image):
        image = PIL.Image.fromarray(image)
    image, depthmap, intrinsics, additional_quantities = rescale_image_and_other_optional_info(
        image=image, output_resolution=np.array(resolution), depthmap=depthmap, camera_intrinsics=intrinsics,
        additional_quantities_to_be_resized_with_nearest=additional_quantities)
    if intrinsics is not None:
        new_intrinsics = camera_matrix_of_crop(intrinsics, image.size, resolution, offset_factor=0.5)
        crop_bbox = bbox_from_intrinsics_in_out(intrinsics, new_intrinsics, resolution)
    else:
        w, h = image.size
        target_w, target_h = resolution
        left, top = (w - target_w) // 2, (h - target_h) // 2
        crop_bbox = (left, top, left + target_w, top + target_h)
    image, depthmap, new_intrinsics, additional_quantities = crop_image_and_other_optional_info(
        image=image, crop_bbox=crop_bbox, depthmap=depthmap, camera_intrinsics=intrinsics,
        additional_quantities=additional_quantities)
    out = (image,)
    if depthmap is not None:
        out += (depthmap,)
    if new_intrinsics is not None:
        out += (new_intrinsics,)
    if additional_quantities is not None:
        out += (additional_quantities,)
    return out

"""Host half of the GPU resize (include/mapa.h mapa_resize_plan_build, csrc/resample.hip): the fixed-point weight
plan, run through a numpy statement of the two integer passes the kernels execute, is bit-identical with PIL's
Image.resize (the reference's resampler, cropping.py:188-280) on noise images, every filter the reference uses,
up- and down-scales, one-pass cases and crops.  No device needed (the plan is host code)."""
import numpy as np
import PIL.Image
import pytest

import conftest  # noqa: F401  (package path)
from mapanything import _native as nat

PIL_FILTER = {1: PIL.Image.Resampling.LANCZOS, 2: PIL.Image.Resampling.BILINEAR, 3: PIL.Image.Resampling.BICUBIC}


def passes(src: np.ndarray, blob) -> np.ndarray:
    """The kernels' arithmetic (resample.hip resize_h_kernel / resize_v_kernel) on the whole resized image, then the
    crop: acc = 2^21 + sum(u8 * w) (no int32 overflow possible: |sum w| < 2^23 / 255), clip8(acc >> 22) per pass."""
    h = nat.resize_plan_header(blob)
    x = src.astype(np.int64)
    for axis, need, n_out, k, ob, ok in ((1, h.need_h, h.rs_w, h.kh, h.off_hb, h.off_hk),
                                         (0, h.need_v, h.rs_h, h.kv, h.off_vb, h.off_vk)):
        if not need:
            continue
        b = blob[ob:ob + 2 * n_out].reshape(n_out, 2).astype(np.int64)
        w = blob[ok:ok + n_out * k].reshape(n_out, k).astype(np.int64)
        assert np.all(w[np.arange(k)[None, :] >= b[:, 1:2]] == 0)  # weights past the window are zero
        idx = np.minimum(b[:, 0:1] + np.arange(k)[None, :], x.shape[axis] - 1)
        if axis == 1:
            acc = np.einsum("hwtc,wt->hwc", x[:, idx, :], w)
        else:
            acc = np.einsum("htwc,ht->hwc", x[idx, :, :], w)
        x = np.clip((acc + (1 << 21)) >> 22, 0, 255)
    return x[h.crop_top:h.crop_top + h.out_h, h.crop_left:h.crop_left + h.out_w].astype(np.uint8)


CASES = [  # (in_w, in_h, rs_w, rs_h, crop (l, t, w, h) or None, filter)
    (1024, 1024, 518, 518, None, 1),          # the bench's from-files source
    (1920, 1080, 522, 294, (2, 0, 518, 294), 1),  # 16:9 -> fixed_mapping 518x294 (centre crop)
    (640, 480, 700, 525, (91, 7, 518, 392), 3),   # upscale (bicubic) + crop
    (300, 200, 300, 150, None, 1),             # vertical pass only
    (300, 200, 150, 200, None, 3),             # horizontal pass only
    (5, 3, 518, 311, (0, 3, 518, 294), 3),     # extreme upscale
    (1000, 700, 6, 5, None, 1),                # extreme downscale (166x: 1001-tap windows)
    (333, 517, 97, 251, (3, 5, 90, 240), 2),   # bilinear, odd sizes
    (64, 48, 64, 48, (4, 2, 56, 42), 1),       # no resize: plain crop (PIL copies)
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}x{c[1]}-{c[2]}x{c[3]}-f{c[5]}")
def test_plan_passes_match_pil(case):
    in_w, in_h, rs_w, rs_h, crop, f = case
    crop = crop or (0, 0, rs_w, rs_h)
    rng = np.random.default_rng(in_w * 7919 + in_h)
    src = rng.integers(0, 256, (in_h, in_w, 3), dtype=np.uint8)
    if in_w >= 256:  # smooth + noise: exercises both the clipping and the in-range rounding
        yy, xx = np.mgrid[0:in_h, 0:in_w]
        src = ((np.sin(xx / 37.0) * np.cos(yy / 23.0) * 100 + 128)[..., None] + rng.normal(0, 30, (in_h, in_w, 3)))
        src = np.clip(src, 0, 255).astype(np.uint8)
    blob = nat.resize_plan(in_w, in_h, rs_w, rs_h, *crop, f)
    h = nat.resize_plan_header(blob)
    assert (h.need_h, h.need_v) == (rs_w != in_w, rs_h != in_h)
    ref = PIL.Image.fromarray(src).resize((rs_w, rs_h), resample=PIL_FILTER[f])
    ref = np.asarray(ref.crop((crop[0], crop[1], crop[0] + crop[2], crop[1] + crop[3])))
    got = passes(src, blob)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), f"{int((got != ref).sum())} channel values differ"


def test_plan_rows_cover_the_crop():
    """row0 / nrows: exactly the input rows the kept output rows' vertical windows read."""
    blob = nat.resize_plan(1920, 1080, 522, 294, 2, 10, 518, 200, 1)
    h = nat.resize_plan_header(blob)
    b = blob[h.off_vb:h.off_vb + 2 * h.rs_h].reshape(-1, 2)
    rows = b[10:210]
    assert h.row0 == rows[:, 0].min() and h.row0 + h.nrows == (rows[:, 0] + rows[:, 1]).max()
    assert nat.resize_workspace_bytes(blob) == 4 * h.nrows * 518


@pytest.mark.parametrize("bad", [
    dict(crop_left=10, out_w=518),        # crop past the resized width
    dict(filter_=0),                      # NEAREST is not a windowed filter
    dict(rs_w=0),
])
def test_plan_rejects_bad_arguments(bad):
    a = dict(in_w=1024, in_h=1024, rs_w=518, rs_h=518, crop_left=0, crop_top=0, out_w=518, out_h=518, filter_=1)
    a.update(bad)
    with pytest.raises(nat.NativeError):
        nat.resize_plan(**a)

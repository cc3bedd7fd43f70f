"""infer() post-processing masks (inference.py:407-506) against fixtures of the REAL reference
(tests/golden/make_postprocess_golden.py on the seeded scenes of tests/golden/postprocess_cases.py).

Boolean work, so the bar is bit-exact: the CPU oracle's numpy restatement (oracle/mapa_oracle.py) and the HIP
kernels (mapa_postprocess_mask + mapa_apply_mask + mapa_confidence_mask) must both reproduce every mask bit of
the reference, for every option set (edge masks on/off, thresholds, confidence percentile), including views with
NaN points, zero depths, border strips and an all-False view.
"""

import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import postprocess_cases as pc  # noqa: E402


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLDEN, "golden_postprocess.npz")) as z:
        return {k: z[k] for k in z.files}


def _ref_mask(gold, name, oi, shape):
    bits = np.unpackbits(gold[f"{name}_{pc.option_key(oi)}_mask"])
    return bits[: int(np.prod(shape))].reshape(shape).astype(bool)


@pytest.mark.parametrize("name", list(pc.CASES))
def test_oracle_mask_matches_reference(gold, name):
    from oracle.mapa_oracle import postprocess_mask_np

    sc = pc.make_scene(pc.CASES[name])
    for oi, opt in enumerate(pc.OPTIONS):
        m = postprocess_mask_np(sc["pts3d"], sc["pts3d_cam"][..., 2], sc["non_ambiguous_mask"],
                                torch.from_numpy(sc["conf"]), **opt)
        ref = _ref_mask(gold, name, oi, m.shape)
        assert np.array_equal(m, ref), (name, oi, int((m != ref).sum()))


def test_normal_threshold_is_numpy_arccos_boundary():
    from mapanything.utils.inference import normal_cos_threshold

    for tol in (5.0, 2.0, 30.0, 0.5, 89.0, 90.0, 179.0):
        c = np.float32(normal_cos_threshold(tol))
        # every float32 within 4096 ulps of the boundary classifies like numpy's arccos against deg2rad(tol)
        base = c.view(np.int32)
        ks = np.arange(-4096, 4096, dtype=np.int64) + int(base)
        ds = ks.astype(np.int32).view(np.float32)
        ds = ds[(ds >= -1) & (ds <= 1) & (ds > 0 if c > 0 else True)]
        assert np.array_equal(np.arccos(ds).astype(np.float64) > np.deg2rad(tol), ds < c), tol
    assert normal_cos_threshold(-1.0) == 2.0 and normal_cos_threshold(181.0) == -1.0


def test_library_threshold_agrees_at_default():
    """The C-ABI helper (double arccos) gives the same boundary as numpy at the reference's default 5 deg."""
    from mapanything import _native as nat
    from mapanything.utils.inference import normal_cos_threshold

    for tol in (5.0, 2.0, 30.0):
        assert nat.normal_cos_threshold(tol) == normal_cos_threshold(tol)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(pc.CASES))
def test_gpu_postprocess_matches_reference(gold, name):
    from mapanything.utils.inference import postprocess_outputs

    case = pc.CASES[name]
    sc = pc.make_scene(case)
    V, H, W = case["views"], case["h"], case["w"]
    dev = torch.device("cuda")
    mean = torch.tensor(pc.MEAN, device=dev)
    std = torch.tensor(pc.STD, device=dev)
    imgs = torch.from_numpy(sc["img"]).to(dev)
    for oi, opt in enumerate(pc.OPTIONS):
        raw = {k: torch.from_numpy(sc[k].copy()).to(dev) for k in
               ("pts3d", "pts3d_cam", "ray_directions", "depth_along_ray", "conf", "non_ambiguous_mask")}
        post = postprocess_outputs(raw, imgs, mean, std, apply_mask=True, **opt)
        torch.cuda.synchronize()
        m = post["mask"].cpu().numpy()
        ref = _ref_mask(gold, name, oi, (V, H, W))
        assert np.array_equal(m, ref), (name, oi, int((m != ref).sum()))
        # geometry zeroing: x * mask, bit for bit (NaN * 0 = NaN, -x * 0 = -0)
        for k in ("pts3d", "pts3d_cam", "depth_along_ray"):
            exp = sc[k] * ref.reshape(V, H, W, 1).astype(np.float32)
            got = post[k].cpu().numpy()
            assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (name, oi, k)
        if name == "pp_small":
            for k in ("pts3d", "depth_along_ray"):
                g = gold[f"{name}_{pc.option_key(oi)}_{k}"]
                assert np.array_equal(post[k].cpu().numpy().view(np.uint32), g.view(np.uint32)), (oi, k)
        if oi == 0:
            if f"{name}_img_no_norm" in gold:
                assert np.array_equal(post["img_no_norm"].cpu().numpy(), gold[f"{name}_img_no_norm"])
            np.testing.assert_allclose(post["intrinsics"].cpu().numpy(), gold[f"{name}_intrinsics"], rtol=2e-5,
                                       atol=1e-3)

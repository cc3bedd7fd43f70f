"""GPU resize kernels (csrc/resample.hip, mapa_resize_normalize) bit-exact with PIL's Image.resize + crop on the
plan cases of test_resample_plan (every filter the reference uses, one-pass cases, extreme scales, crops), for both
outputs: the 8-bit image and the normalised float32 planes (torchvision's ToTensor + Normalize order)."""
import numpy as np
import PIL.Image
import pytest
import torch

import conftest  # noqa: F401  (package path)
from mapanything import _native as nat
from test_resample_plan import CASES, PIL_FILTER

pytestmark = pytest.mark.gpu

MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


def _src(in_w, in_h):
    rng = np.random.default_rng(in_w * 7919 + in_h)
    return rng.integers(0, 256, (in_h, in_w, 3), dtype=np.uint8)


@pytest.mark.parametrize("pad", [0, 13], ids=["packed", "row_pad"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}x{c[1]}-{c[2]}x{c[3]}-f{c[5]}")
def test_resize_normalize_matches_pil(case, pad):
    in_w, in_h, rs_w, rs_h, crop, f = case
    crop = crop or (0, 0, rs_w, rs_h)
    src = _src(in_w, in_h)
    ref = PIL.Image.fromarray(src).resize((rs_w, rs_h), resample=PIL_FILTER[f])
    ref = np.asarray(ref.crop((crop[0], crop[1], crop[0] + crop[2], crop[1] + crop[3])))
    blob = nat.resize_plan(in_w, in_h, rs_w, rs_h, *crop, f)
    ld = 3 * in_w + pad  # rows of a larger (strided) buffer
    host = np.zeros((in_h, ld), np.uint8)
    host[:, :3 * in_w] = src.reshape(in_h, -1)
    d = torch.from_numpy(host).cuda()
    plan = torch.from_numpy(blob).cuda()
    ws = torch.empty(max(nat.resize_workspace_bytes(blob), 1), dtype=torch.uint8, device="cuda")
    out = torch.empty(3, crop[3], crop[2], device="cuda")
    out_u8 = torch.empty(crop[3], crop[2], 3, dtype=torch.uint8, device="cuda")
    nat.resize_normalize(d, ld, blob, plan, MEAN, STD, out=out, out_u8=out_u8, workspace=ws)
    torch.cuda.synchronize()
    got = out_u8.cpu().numpy()
    assert np.array_equal(got, ref), f"{int((got != ref).sum())} channel values differ from PIL"
    # float planes: torchvision's ToTensor (x / 255) then Normalize ((x - mean) / std), float32 per operation
    t = torch.from_numpy(ref).permute(2, 0, 1).float().div(255)
    t = (t - torch.tensor(MEAN)[:, None, None]) / torch.tensor(STD)[:, None, None]
    assert torch.equal(out.cpu(), t)


def test_resize_normalize_rejects_short_workspace():
    blob = nat.resize_plan(1024, 1024, 518, 518, 0, 0, 518, 518, nat.RESAMPLE_LANCZOS)
    d = torch.zeros(1024, 3072, dtype=torch.uint8, device="cuda")
    plan = torch.from_numpy(blob).cuda()
    out = torch.empty(3, 518, 518, device="cuda")
    ws = torch.empty(16, dtype=torch.uint8, device="cuda")
    with pytest.raises(nat.NativeError):
        nat.resize_normalize(d, 3072, blob, plan, MEAN, STD, out=out, workspace=ws)

"""TF32-equivalent head operands (include/mapa.h MAPA_F16X2) through every kernel path the heads use (needs an MI355X).

The reference runs its heads with autocast disabled (model.py:1774), i.e. as fp32 convs / linears, which its own GPUs
execute in TF32 (cudnn's default; `torch.backends.cuda.matmul.allow_tf32 = True` at model.py:93): both operands
rounded to 11 significant bits, fp32 accumulation.  Here activations are stored as binary16 [hi | lo]
(hi = f16(x), lo = f16(x - hi): 22 bits) and weights as f16 [w | w], and one f16 MFMA GEMM over K = 2C accumulates
w*(x_hi + x_lo).  Each test checks the library against a float64 conv / linear with the weights rounded to f16 —
the exact arithmetic the scheme promises, to fp32 accumulation order (<= 2e-5 rel-L2) — and against the unrounded
float64 result at TF32 level (<= 1e-3)."""

import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    from mapanything import _native

    _native.lib()
    return _native


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).cuda()


def _conv_weight(wt, kblock=32):
    """[Co][C][3][3] fp32 -> f16 [Co][9 * 2C] = [w | w] per tap, in the channel-block-major K order when kblock."""
    Co, C = wt.shape[:2]
    wk = wt.permute(0, 2, 3, 1).reshape(Co, 9, C).to(torch.float16)
    wp = torch.cat([wk, wk], 2)  # [out][tap][2C]
    if kblock:
        wp = wp.reshape(Co, 9, 2 * C // kblock, kblock).permute(0, 2, 1, 3)
    wp = wp.contiguous().reshape(Co, -1)
    wp._mapa_split = True
    if kblock:
        wp._mapa_kblock = kblock
    return wp


def _split(nat, x2d):
    M, C = x2d.shape
    a = torch.empty(M, 2 * C, dtype=torch.float16, device="cuda")
    nat.split_rows(x2d.contiguous(), M, C, C, a)
    return a


def _refs(x, wt, stride=1):
    """(float64 conv with f16-rounded weights, float64 conv), NHWC rows."""
    xd = x.cpu().double()
    r16 = F.conv2d(xd, wt.to(torch.float16).cpu().double(), padding=1, stride=stride)
    r = F.conv2d(xd, wt.cpu().double(), padding=1, stride=stride)
    Co = wt.shape[0]
    return (r16.permute(0, 2, 3, 1).reshape(-1, Co), r.permute(0, 2, 3, 1).reshape(-1, Co))


def test_split_rows_f16x2_is_22_bits(nat):
    x = _rand(1000, 96, scale=7.0, seed=1)
    a = _split(nat, x)
    hi, lo = a[:, :96].float(), a[:, 96:].float()
    assert torch.equal(hi, x.half().float())
    assert (hi + lo - x).abs().max().item() <= x.abs().max().item() * 2.0 ** -21


# variant codes (mapa_gemm_set_variant): 0 automatic; 2584 / 2588 halo-window conv (128-wide 16-row / 256-wide 8-row
# blocks); 2589 flat-raster split-K halo; 2568 / 2571 / 2574 implicit-GEMM tiles; 643 the 128-row kernel;
# 2581 stream-K
@pytest.mark.parametrize("variant,n,h,w,C,Co", [
    (0, 2, 40, 40, 256, 256), (2584, 2, 37, 41, 64, 128), (2588, 1, 33, 30, 96, 256), (2588, 1, 34, 29, 64, 256),
    (2589, 3, 19, 19, 256, 256), (2568, 2, 21, 23, 64, 256), (2571, 2, 21, 23, 64, 128), (2574, 2, 20, 20, 64, 256),
    (643, 1, 13, 11, 32, 64), (2581, 2, 19, 19, 768, 256)])
def test_f16x2_conv3x3_paths(nat, variant, n, h, w, C, Co):
    x = _rand(n, C, h, w, seed=2)
    wt = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=3)
    b = _rand(Co, seed=4)
    r16, r = _refs(x, wt)
    a = _split(nat, x.permute(0, 2, 3, 1).reshape(-1, C))
    kb = 0 if variant in (643,) else 32
    wp = _conv_weight(wt, kb)
    M = n * h * w
    out = torch.empty(M, Co, device="cuda")
    s3 = torch.empty(M, 2 * Co, dtype=torch.float16, device="cuda")
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(a, wp, M, Co, 9 * 2 * C, bias=b, out_f32=out, out_s3=s3, conv=(2 * C, h, w, h, w, 1))
    finally:
        nat.gemm_set_variant(0)
    ref16 = r16 + b.cpu().double()
    assert rel_l2(out.cpu(), ref16) < 2e-5
    assert rel_l2(out.cpu(), r + b.cpu().double()) < 1e-3
    # the split output is the fp32 output to 22 bits
    v = s3[:, :Co].float() + s3[:, Co:].float()
    assert rel_l2(v.cpu(), out.cpu()) < 1e-6


def test_f16x2_stride2_conv_streamk(nat):
    n, h, w, C, Co = 2, 37, 37, 768, 768
    x = _rand(n, C, h, w, seed=5)
    wt = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=6)
    r16, r = _refs(x, wt, stride=2)
    a = _split(nat, x.permute(0, 2, 3, 1).reshape(-1, C))
    oh, ow = 19, 19
    out = torch.empty(n * oh * ow, Co, device="cuda")
    nat.gemm(a, _conv_weight(wt), n * oh * ow, Co, 9 * 2 * C, out_f32=out, conv=(2 * C, h, w, oh, ow, 2))
    assert rel_l2(out.cpu(), r16) < 2e-5
    assert rel_l2(out.cpu(), r) < 1e-3


@pytest.mark.parametrize("M,N,K", [(10952, 784, 784), (2888, 256, 768), (300, 96, 1024), (10952, 1536, 96)])
def test_f16x2_linear_and_relu_split_outputs(nat, M, N, K):
    x = _rand(M, K, seed=7)
    wt = _rand(N, K, scale=K ** -0.5, seed=8)
    b = _rand(N, seed=9)
    a = _split(nat, x)
    w16 = wt.half()
    wp = torch.cat([w16, w16], 1).contiguous()
    wp._mapa_split = True
    out = torch.empty(M, N, device="cuda")
    s3r = torch.empty(M, 2 * N, dtype=torch.float16, device="cuda")
    nat.gemm(a, wp, M, N, 2 * K, bias=b, act=nat.ACT_RELU, out_f32=out, out_s3_relu=s3r)
    ref16 = torch.relu(x.cpu().double() @ w16.cpu().double().t() + b.cpu().double())
    assert rel_l2(out.cpu(), ref16) < 2e-5
    v = s3r[:, :N].float() + s3r[:, N:].float()
    assert rel_l2(v.cpu(), torch.relu(out).cpu()) < 1e-6


def test_f16x2_pixel_shuffle(nat):
    """ConvTranspose k = s = 4 as a GEMM with the pixel-shuffle epilogue writing split rows."""
    n, hp, wp_, ci, co, s = 2, 7, 9, 96, 96, 4
    x = _rand(n, ci, hp, wp_, seed=10)
    wt = _rand(ci, co, s, s, scale=ci ** -0.5, seed=11)
    b = _rand(co, seed=12)
    a = _split(nat, x.permute(0, 2, 3, 1).reshape(-1, ci))
    wk = wt.permute(2, 3, 1, 0).reshape(s * s * co, ci).half()
    wp = torch.cat([wk, wk], 1).contiguous()
    wp._mapa_split = True
    out = torch.empty(n * hp * s * wp_ * s, 2 * co, dtype=torch.float16, device="cuda")
    nat.gemm(a, wp, n * hp * wp_, s * s * co, 2 * ci, bias=b, bias_mod=co, pixshuf=(s, hp, wp_, co), out_s3=out)
    ref = F.conv_transpose2d(x.cpu().double(), wt.half().cpu().double(), b.cpu().double(), stride=s)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, co)
    v = out[:, :co].float() + out[:, co:].float()
    assert rel_l2(v.cpu(), ref) < 2e-5


def test_f16x2_layernorm_and_bilinear_outputs(nat):
    rows, dim = 777, 768
    x = _rand(rows, dim, scale=3.0, seed=13) + 5.0
    w, b = _rand(dim, seed=14), _rand(dim, seed=15)
    y = torch.empty(rows, 2 * dim, dtype=torch.float16, device="cuda")
    nat.layernorm(x, rows, dim, w, b, y_s3=y)
    ref = F.layer_norm(x.double(), (dim,), w.double(), b.double(), eps=1e-6)
    assert rel_l2((y[:, :dim].float() + y[:, dim:].float()).cpu(), ref.cpu()) < 1e-6
    n, IH, IW, C, O = 2, 37, 41, 128, 64
    src = _rand(n, IH, IW, C, seed=16)
    out = torch.empty(n * O * O, 2 * C, dtype=torch.float16, device="cuda")
    nat.bilinear_ac(src, n, IH, IW, C, O, O, O, O, out, split_out=True)
    f32 = torch.empty(n * O * O, C, device="cuda")
    nat.bilinear_ac(src, n, IH, IW, C, O, O, O, O, f32)
    assert rel_l2((out[:, :C].float() + out[:, C:].float()).cpu(), f32.cpu()) < 1e-6


def test_f16x2_range_fault_raises(nat):
    """A value outside binary16's range sets MAPA_FAULT_F16_RANGE (sticky, read and reset by check_faults)."""
    nat.fault_status(reset=True)
    x = _rand(64, 32, seed=17)
    x[5, 7] = 1.0e5
    _split(nat, x)
    torch.cuda.synchronize()
    with pytest.raises(nat.NativeError, match="F16_RANGE"):
        nat.check_faults()
    assert nat.fault_status(reset=True) == 0
    _split(nat, _rand(64, 32, seed=18))
    nat.check_faults()  # in range: nothing raised


@pytest.mark.parametrize("n,H,W", [(2, 70, 51), (1, 518, 518)])
def test_f16x2_regressor_head_out_fused(nat, n, H, W):
    """The regressor's conv2 carrying the dense head (mapa_regressor_head_out) on TF32-equivalent operands against
    the two-launch path (conv out_f32 + mapa_dense_head_out) on the same operands: same f16 MFMA products, other fp32
    summation order."""
    C = 128
    x = _rand(n, C, H, W, seed=60).relu()
    wt = _rand(C, C, 3, 3, scale=(9 * C) ** -0.5, seed=61)
    b2, w6, b6 = _rand(C, seed=62), _rand(6, C, scale=C ** -0.5, seed=63), _rand(6, seed=64)
    M = n * H * W
    a = _split(nat, x.permute(0, 2, 3, 1).reshape(M, C))
    wp = _conv_weight(wt)
    pose_out = torch.empty(n, 19, device="cuda")
    scale = torch.empty(1, device="cuda")
    nat.pose_scale_finalize(_rand(n, 7, seed=65), _rand(1, seed=66), n, 1, pose_out, scale,
                            torch.empty(n, 4, 4, device="cuda"))

    def outs():
        f = dict(device="cuda")
        return [torch.full((n, H, W, 3), float("nan"), **f) for _ in range(3)] + \
            [torch.full((n, H, W, 1), float("nan"), **f)] + [torch.full((n, H, W), float("nan"), **f) for _ in range(2)] + \
            [torch.full((n, H, W), 7, dtype=torch.uint8, device="cuda")]

    conv = (2 * C, H, W, H, W, 1)
    hid = torch.empty(M, C, device="cuda")
    nat.gemm(a, wp, M, C, 9 * 2 * C, bias=b2, act=nat.ACT_RELU, out_f32=hid, conv=conv)
    ref = outs()
    nat.dense_head_out(hid, n, H * W, w6, b6, pose_out, scale, 1, *ref)
    got = outs()
    nat.gemm(a, wp, M, C, 9 * 2 * C, bias=b2, act=nat.ACT_RELU, conv=conv, head_out=(w6, b6, pose_out, scale, n, *got))
    torch.cuda.synchronize()
    for r, g in zip(ref[:6], got[:6]):
        assert torch.isfinite(g).all()
        assert rel_l2(g.cpu(), r.cpu()) < 1e-5
    sure = ref[5].abs() > 1e-4
    assert torch.equal(got[6][sure], ref[6][sure])


# ------------------------------------------------------------------ plain binary16 operands (head_precision="tf32")
def _tf32(t):
    """TF32 rounding of fp32 values (10 explicit mantissa bits, round to nearest even), in float64."""
    b = t.float().contiguous().view(torch.int32).to(torch.int64)
    lsb = (b >> 13) & 1
    r = ((b + 0xFFF + lsb) & ~0x1FFF) & 0xFFFFFFFF
    r = torch.where(r >= 2 ** 31, r - 2 ** 32, r).to(torch.int32)
    return r.view(torch.float32).double()


@pytest.mark.parametrize("variant,n,h,w,C,Co", [
    (0, 2, 40, 40, 256, 256), (2584, 2, 37, 41, 64, 128), (2588, 1, 33, 30, 96, 256), (2589, 3, 19, 19, 256, 256),
    (2574, 2, 20, 20, 64, 256), (643, 1, 13, 11, 32, 64), (2581, 2, 19, 19, 768, 256)])
def test_f16_conv3x3_is_the_tf32_product(nat, variant, n, h, w, C, Co):
    """binary16 activations x binary16 weights (the TF32-equivalent heads): the float64 conv of the TF32-rounded
    operands — the reference's own TF32 arithmetic on its GPUs — to fp32 accumulation order (<= 2e-5)."""
    x = _rand(n, C, h, w, seed=20)
    wt = _rand(Co, C, 3, 3, scale=(9 * C) ** -0.5, seed=21)
    b = _rand(Co, seed=22)
    ref = F.conv2d(_tf32(x).cpu(), _tf32(wt).cpu(), padding=1) + b.cpu().double()[None, :, None, None]
    ref = ref.permute(0, 2, 3, 1).reshape(-1, Co)
    M = n * h * w
    a = torch.empty(M, C, dtype=torch.float16, device="cuda")
    nat.convert_rows(x.permute(0, 2, 3, 1).reshape(M, C).contiguous(), C, M, C, a, C)
    kb = 0 if variant == 643 else 32
    wk = wt.permute(0, 2, 3, 1).reshape(Co, 9, C).half()
    if kb:
        wk = wk.reshape(Co, 9, C // kb, kb).permute(0, 2, 1, 3)
    wp = wk.contiguous().reshape(Co, -1)
    wp._mapa_split = True
    if kb:
        wp._mapa_kblock = kb
    out = torch.empty(M, Co, device="cuda")
    lp = torch.empty(M, Co, dtype=torch.float16, device="cuda")
    nat.gemm_set_variant(variant)
    try:
        nat.gemm(a, wp, M, Co, 9 * C, bias=b, out_f32=out, out_lp=lp, conv=(C, h, w, h, w, 1))
    finally:
        nat.gemm_set_variant(0)
    assert rel_l2(out.cpu(), ref) < 2e-5
    assert torch.equal(lp, out.half())


def test_f16_bilinear_and_convert_rows_range_faults(nat):
    n, IH, IW, C, O = 2, 37, 41, 128, 64
    src = _rand(n, IH, IW, C, seed=23)
    out = torch.empty(n * O * O, C, dtype=torch.float16, device="cuda")
    nat.bilinear_ac(src, n, IH, IW, C, O, O, O, O, out)
    f32 = torch.empty(n * O * O, C, device="cuda")
    nat.bilinear_ac(src, n, IH, IW, C, O, O, O, O, f32)
    assert torch.equal(out, f32.half())
    nat.check_faults()
    src[1, 3, 4, 5] = 1.0e6  # every output pixel it feeds leaves the range
    nat.bilinear_ac(src, n, IH, IW, C, O, O, O, O, out)
    with pytest.raises(nat.NativeError, match="F16_RANGE"):
        nat.check_faults()
    x = _rand(50, 40, seed=24)
    y = torch.empty(50, 40, dtype=torch.float16, device="cuda")
    nat.convert_rows(x, 40, 50, 40, y, 40)
    nat.check_faults()
    x[3, 3] = -1.0e6
    nat.convert_rows(x, 40, 50, 40, y, 40)
    with pytest.raises(nat.NativeError, match="F16_RANGE"):
        nat.check_faults()

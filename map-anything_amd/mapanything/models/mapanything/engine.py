"""Device executor of the MapAnything feed-forward path on MI355X (every op is a libmapa.so HIP kernel).

`MapaEngine.run(imgs)` is the GPU replacement of `MapAnything.forward` (model.py:1657-2152) for the released
config (image-only inputs, pred head "dpt+pose", scene rep "raydirs+depth+pose+confidence+mask").  Tensors are
torch allocations on the current device; torch does nothing else.  Layout in HBM:

  tokens            row-major [rows][C]: encoder rows = view*(T+1) + t (cls first), AAT rows = view*T + t with the
                    scale token as the last row; residual streams fp32, GEMM operands bf16 (fp32 in precise mode)
  qkv               one [rows][3*C] buffer straight from the qkv GEMM; attention reads q/k/v in place
  DPT feature maps  NHWC [view][y][x][C]; 3x3 convs are implicit GEMMs over these, ConvTranspose k=s writes the
                    pixel-shuffled map directly from the GEMM epilogue
  outputs           NHWC fp32 [view][H][W][c] (the reference's (B,H,W,c) per view, view-major)

Precision modes: "bf16" (the reference's own autocast recipe, model.py:2287-2302: the encoder and the transformer run
on bf16 MFMA operands with fp32 accumulate / LayerNorm / softmax / residuals; "fp16" the same on fp16 operands —
infer(amp_dtype="fp16"); the geometric-input encoders
(autocast disabled, model.py:1377) and the downstream heads (autocast disabled, model.py:1774-1799) stay fp32-exact,
computed as split-precision bf16 GEMMs: activations [hi | hi | lo], weights [hi | lo | hi], ~2^-16 relative) and
"fp32" (exact-fp32 MFMA everywhere, for parity against the fp32 reference to ~1e-5).  heads="bf16" is an opt-in
fast mode that runs the heads on plain bf16 operands — NOT the reference's recipe (bench.py reports it as a
separate, labelled line).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from ... import _native as nat
from ...parallel import force_collectives, force_overlap
from .spec import RELEASED_INFO, InfoSharingSpec

ENC_DIM, ENC_HEADS, PATCH, KPAD = 1024, 16, 14, 640
AAT_DIM, AAT_HEADS = 768, 12  # the released transformer; variants carry their own (InfoSharingSpec)
POSE_DIM = 784
LN_EPS = 1e-6
DINOV2_MEAN = (0.485, 0.456, 0.406)
DINOV2_STD = (0.229, 0.224, 0.225)


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().float().cpu().numpy()
    return np.asarray(x, dtype=np.float32)


@dataclass
class GeoInputs:
    """Optional geometric inputs of this rank's views, prepared by MapAnything (model.py:1292-1438 with the
    deterministic masks of infer(), model.py:2154-2197).  Dense inputs hold every local view (zeros where the
    view has no such input, as the reference builds them); the *_views lists are the views whose mask is set.
    Camera arrays cover ALL views (translation normalisation is across views), local views start at local_start."""
    rays: Optional[torch.Tensor] = None          # (n_local, H, W, 3) f32
    ray_views: List[int] = field(default_factory=list)
    depth: Optional[torch.Tensor] = None         # (n_local, H, W) f32 depth along ray
    depth_views: List[int] = field(default_factory=list)
    depth_metric: List[bool] = field(default_factory=list)   # per local view (is_metric_scale & use_depth_scale)
    cam_quats: Optional[torch.Tensor] = None     # (V, 4) f32, (x, y, z, w)
    cam_trans: Optional[torch.Tensor] = None     # (V, 3) f32
    cam_mask: List[bool] = field(default_factory=list)       # (V,)
    pose_metric: List[bool] = field(default_factory=list)    # (V,) is_metric_scale & use_pose_scale
    local_start: int = 0
    # B > 1 batched scenes: every list / tensor above holds the B scenes' views scene-major (dense inputs: local image
    # b*n_local + i; camera arrays: view b*V + v); the camera translations are normalised per scene (pose inputs over
    # each scene's V views, model.py:792-896)
    scenes: int = 1

    def empty(self) -> bool:
        return not self.ray_views and not self.depth_views and not any(self.cam_mask)

    def signature(self) -> tuple:
        """The host-side structure (which views carry which input, the metric flags): the HIP-graph key of a
        geometric forward — the tensors are refreshed into the graph's static copies before every replay."""
        shp = lambda t: None if t is None else tuple(t.shape)  # noqa: E731
        return (tuple(self.ray_views), tuple(self.depth_views), tuple(self.depth_metric), tuple(self.cam_mask),
                tuple(self.pose_metric), self.local_start, self.scenes, shp(self.rays), shp(self.depth),
                shp(self.cam_quats), shp(self.cam_trans))

    def tensors(self):
        return ("rays", "depth", "cam_quats", "cam_trans")

    def static_copy(self) -> "GeoInputs":
        """The same inputs in fresh buffers (a captured graph's static inputs)."""
        import copy

        g = copy.copy(self)
        for k in self.tensors():
            t = getattr(self, k)
            setattr(g, k, None if t is None else t.clone())
        return g

    def refresh_into(self, static: "GeoInputs"):
        for k in self.tensors():
            t = getattr(self, k)
            if t is not None:
                getattr(static, k).copy_(t)


KBLOCK = 32  # channel block of the head convs' K order (include/mapa.h conv_kblock)


# A binary16 head weight whose largest magnitude lies in [2^WS_LO, 2^WS_HI] is stored as is; otherwise it is stored
# as 2^s x w with s putting that magnitude in [2^8, 2^9) (_f16_wscale), and the GEMM epilogue takes the power of two
# back out exactly (_native._wscale_epilogue).  TF32 has fp32's 8-bit exponent: a weight tensor of tiny (or huge)
# values keeps its 11 significant bits there, and keeps them here too.
WS_LO, WS_HI = -4, 12


def _f16_wscale(wt: torch.Tensor) -> int:
    """Power-of-two exponent s of a binary16 weight's storage scale (0 = stored as is)."""
    m = float(wt.abs().max()) if wt.numel() else 0.0
    if m == 0.0 or 2.0 ** WS_LO <= m <= 2.0 ** WS_HI:
        return 0
    return 8 - math.floor(math.log2(m))


def _f16_pack(w: np.ndarray, dev, scaled: bool = False) -> torch.Tensor:
    """[out][taps][cin] fp32 -> binary16 [out][taps * ceil8(cin)]: the weight side of the TF32-equivalent heads
    (activations binary16 too, include/mapa.h MAPA_F16): both operands at TF32's 11 significant bits, fp32
    accumulation, on the f16 MFMA pipe at the bf16 rate.  scaled: store 2^s x w for a weight outside binary16's
    comfortable range (WS_LO / WS_HI; the tensor carries _mapa_wscale = s for nat.gemm's epilogue)."""
    o, taps, cin = w.shape
    wt = torch.from_numpy(np.ascontiguousarray(w)).to(dev)
    s = _f16_wscale(wt) if scaled else 0
    if s:
        wt = wt * (2.0 ** s)
    if bool((wt.abs() > 65504).any()):
        raise ValueError("a head weight exceeds binary16's range: use head_precision='fp32'")
    cp = _ceil8(cin)
    out = torch.zeros(o, taps, cp, dtype=torch.float16, device=dev)
    out[:, :, :cin] = wt.to(torch.float16)
    out = out.reshape(o, -1)
    out._mapa_split = True  # timed with the fp32-recipe heads (nat.gemm: "gemm_split" / "conv3x3_split")
    out._mapa_wscale = s
    return out


def _f16x2_pack(w: np.ndarray, dev, scaled: bool = False) -> torch.Tensor:
    """[out][taps][cin] fp32 -> binary16 [out][taps * 2 * ceil8(cin)] = [w | w] per tap: the weight side of the
    TF32-equivalent heads (activations stored [hi | lo] of binary16, include/mapa.h MAPA_F16X2), a plain f16 GEMM over
    K = 2C that accumulates w*(x_hi + x_lo): the weight at 11 significant bits as TF32 rounds it, the activation at 22.
    scaled: as _f16_pack."""
    o, taps, cin = w.shape
    wt = torch.from_numpy(np.ascontiguousarray(w)).to(dev)
    s = _f16_wscale(wt) if scaled else 0
    if s:
        wt = wt * (2.0 ** s)
    if bool((wt.abs() > 65504).any()):
        raise ValueError("a head weight exceeds binary16's range: use head_precision='fp32'")
    h = wt.to(torch.float16)
    cp = _ceil8(cin)
    out = torch.zeros(o, taps, 2, cp, dtype=torch.float16, device=dev)
    out[:, :, 0, :cin], out[:, :, 1, :cin] = h, h
    out = out.reshape(o, -1)
    out._mapa_split = True  # timed with the split heads (nat.gemm: "gemm_split" / "conv3x3_split")
    out._mapa_wscale = s
    return out


def _split_pack(w: np.ndarray, dev) -> torch.Tensor:
    """[out][taps][cin] fp32 -> bf16 [out][taps * 3 * ceil8(cin)] = [hi | lo | hi] per tap: the weight side of a
    split-precision GEMM against activations stored [hi | lo] and read as [hi | hi | lo] (mapa_split_bf16x3 / the
    GEMM's out_s3 epilogue; nat.gemm sets mapa_gemm_desc.a_split for weights tagged _mapa_split)."""
    o, taps, cin = w.shape
    wt = torch.from_numpy(np.ascontiguousarray(w)).to(dev)
    hi = wt.to(torch.bfloat16)
    lo = (wt - hi.float()).to(torch.bfloat16)
    cp = _ceil8(cin)
    out = torch.zeros(o, taps, 3, cp, dtype=torch.bfloat16, device=dev)
    out[:, :, 0, :cin], out[:, :, 1, :cin], out[:, :, 2, :cin] = hi, lo, hi
    out = out.reshape(o, -1)
    out._mapa_split = True  # timed as its own class (nat.gemm: "gemm_split" / "conv3x3_split")
    return out


class PackedWeights:
    """Canonical state dict -> device buffers in kernel layout (done once at load).  head_split: the downstream
    heads' GEMM weights are packed for split-precision operands (the reference's fp32 heads in bf16 mode)."""

    def __init__(self, sd: Dict[str, object], device, lp_dtype: torch.dtype, info: InfoSharingSpec = RELEASED_INFO,
                 head_split: bool = False, head_fmt: str = "bf16x3"):
        self.device = device
        self.lp = lp_dtype
        self.head_split = head_split
        self.head_fmt = head_fmt
        self.sd = sd
        g = self._get
        dev = device

        def f32(name):
            return torch.from_numpy(np.ascontiguousarray(_np(g(name)))).to(dev)

        def lin(name):
            w = _np(g(f"{name}.weight"))
            return torch.from_numpy(np.ascontiguousarray(w.reshape(w.shape[0], -1))).to(dev, self.lp)

        def conv3(name):  # [co][ci][3][3] -> [co][ky][kx][ci]
            w = _np(g(f"{name}.weight"))
            return torch.from_numpy(np.ascontiguousarray(w.transpose(0, 2, 3, 1).reshape(w.shape[0], -1))).to(
                dev, self.lp)

        def convT(name):  # [ci][co][k][k] -> [(ky*k+kx)*co + c][ci]
            w = _np(g(f"{name}.weight"))
            ci, co, k, _ = w.shape
            return torch.from_numpy(np.ascontiguousarray(w.transpose(2, 3, 1, 0).reshape(k * k * co, ci))).to(
                dev, self.lp)

        def hpack(w):  # head weights [out][taps][cin]: lp (or fp32) [out][taps*cin], or split-packed
            if head_split:  # (binary16 head weights with a power-of-two storage scale where their range needs one)
                if head_fmt in ("f16", "f16x2"):
                    return (_f16_pack if head_fmt == "f16" else _f16x2_pack)(w, dev, scaled=True)
                return _split_pack(w, dev)
            return torch.from_numpy(np.ascontiguousarray(w.reshape(w.shape[0], -1))).to(dev, self.lp)

        def hlin(name):
            w = _np(g(f"{name}.weight"))
            return hpack(w.reshape(w.shape[0], 1, -1))

        def hconv3(name):
            # columns in channel-block-major K order (mapa_gemm_desc.conv_kblock = KBLOCK): [out][C/B][tap][B] of
            # the per-tap (logical, split-packed) channels, so each B-channel slice of the input window stays
            # L2-resident across the 9 taps
            w = _np(g(f"{name}.weight"))
            t = hpack(w.transpose(0, 2, 3, 1).reshape(w.shape[0], 9, w.shape[1]))
            o, c = t.shape[0], t.shape[1] // 9
            if not KBLOCK or c % KBLOCK:
                return t
            r = t.view(o, 9, c // KBLOCK, KBLOCK).permute(0, 2, 1, 3).contiguous().reshape(o, -1)
            r._mapa_split = getattr(t, "_mapa_split", False)
            r._mapa_wscale = getattr(t, "_mapa_wscale", 0)
            r._mapa_kblock = KBLOCK
            return r

        def hconvT(name):
            w = _np(g(f"{name}.weight"))
            ci, co, k, _ = w.shape
            return hpack(w.transpose(2, 3, 1, 0).reshape(k * k * co, 1, ci))

        self.f32, self.lin, self.conv3 = f32, lin, conv3
        # DINOv2
        pe = _np(g("encoder.model.patch_embed.proj.weight")).reshape(ENC_DIM, 588)
        pe = np.concatenate([pe, np.zeros((ENC_DIM, KPAD - 588), np.float32)], 1)
        self.pe_w = torch.from_numpy(np.ascontiguousarray(pe)).to(dev, self.lp)
        self.pe_b = f32("encoder.model.patch_embed.proj.bias")
        self.cls = f32("encoder.model.cls_token").reshape(-1)
        self.pos_embed_param = torch.from_numpy(_np(g("encoder.model.pos_embed")))
        self.pos_cache: Dict[tuple, torch.Tensor] = {}
        self.enc = []
        for b in range(24):
            p = f"encoder.model.blocks.{b}"
            self.enc.append(dict(
                n1w=f32(f"{p}.norm1.weight"), n1b=f32(f"{p}.norm1.bias"),
                qkv=lin(f"{p}.attn.qkv"), qkv_b=f32(f"{p}.attn.qkv.bias"),
                proj=lin(f"{p}.attn.proj"), proj_b=f32(f"{p}.attn.proj.bias"), ls1=f32(f"{p}.ls1.gamma"),
                n2w=f32(f"{p}.norm2.weight"), n2b=f32(f"{p}.norm2.bias"),
                fc1=lin(f"{p}.mlp.fc1"), fc1_b=f32(f"{p}.mlp.fc1.bias"),
                fc2=lin(f"{p}.mlp.fc2"), fc2_b=f32(f"{p}.mlp.fc2.bias"), ls2=f32(f"{p}.ls2.gamma")))
        self.enc_nw, self.enc_nb = f32("encoder.model.norm.weight"), f32("encoder.model.norm.bias")
        self.fus_w, self.fus_b = f32("fusion_norm_layer.weight"), f32("fusion_norm_layer.bias")
        self.scale_token = f32("scale_token")
        # AAT
        # proj_embed is nn.Identity when the transformer is as wide as the encoder (alternating_attention_
        # transformer.py:121-124; the 48-layer configs)
        self.pe_proj = lin("info_sharing.proj_embed") if info.dim != ENC_DIM else None
        self.pe_proj_b = f32("info_sharing.proj_embed.bias") if info.dim != ENC_DIM else None
        # sinusoid view PE table (pe_rows x dim): row 0 = the reference view's, rows 1.. the other views'
        self.view_pos = f32("info_sharing.view_pos_table").reshape(-1, info.dim) if info.ref_pe else None
        self.view_pe = self.view_pos[0].contiguous() if info.ref_pe else None
        self.aat = []
        for b in range(info.depth):
            p = f"info_sharing.self_attention_blocks.{b}"
            self.aat.append(dict(
                n1w=f32(f"{p}.norm1.weight"), n1b=f32(f"{p}.norm1.bias"),
                qkv=lin(f"{p}.attn.qkv"), qkv_b=f32(f"{p}.attn.qkv.bias"),
                proj=lin(f"{p}.attn.proj"), proj_b=f32(f"{p}.attn.proj.bias"),
                n2w=f32(f"{p}.norm2.weight"), n2b=f32(f"{p}.norm2.bias"),
                fc1=lin(f"{p}.mlp.fc1"), fc1_b=f32(f"{p}.mlp.fc1.bias"),
                fc2=lin(f"{p}.mlp.fc2"), fc2_b=f32(f"{p}.mlp.fc2.bias")))
        self.aat_nw, self.aat_nb = f32("info_sharing.norm.weight"), f32("info_sharing.norm.bias")
        # DPT feature head
        h = "dpt_feature_head"
        ip = f"{h}.input_process"
        self.ip = [
            dict(w=hlin(f"{ip}.0.0.0"), b=f32(f"{ip}.0.0.0.bias"), ct=hconvT(f"{ip}.0.0.1"), ct_b=f32(f"{ip}.0.0.1.bias")),
            dict(w=hlin(f"{ip}.1.0.0"), b=f32(f"{ip}.1.0.0.bias"), ct=hconvT(f"{ip}.1.0.1"), ct_b=f32(f"{ip}.1.0.1.bias")),
            dict(w=hlin(f"{ip}.2.0.0"), b=f32(f"{ip}.2.0.0.bias")),
            dict(w=hlin(f"{ip}.3.0.0"), b=f32(f"{ip}.3.0.0.bias"), c3=hconv3(f"{ip}.3.0.1"), c3_b=f32(f"{ip}.3.0.1.bias")),
        ]
        self.layer_rn = [hconv3(f"{h}.scratch.layer{i + 1}_rn") for i in range(4)]
        self.refine = {}
        for r in (1, 2, 3, 4):
            n = f"{h}.scratch.refinenet{r}"
            d = dict(out=hlin(f"{n}.out_conv"), out_b=f32(f"{n}.out_conv.bias"))
            units = ("resConfUnit2",) if r == 4 else ("resConfUnit1", "resConfUnit2")
            for u in units:
                d[u] = dict(c1=hconv3(f"{n}.{u}.conv1"), b1=f32(f"{n}.{u}.conv1.bias"),
                            c2=hconv3(f"{n}.{u}.conv2"), b2=f32(f"{n}.{u}.conv2.bias"))
            self.refine[r] = d
        self.reg_c1, self.reg_b1 = hconv3("dpt_regressor_head.conv1"), f32("dpt_regressor_head.conv1.bias")
        self.reg_c2, self.reg_b2 = hconv3("dpt_regressor_head.conv2.0"), f32("dpt_regressor_head.conv2.0.bias")
        self.reg_w6 = f32("dpt_regressor_head.conv2.2.weight").reshape(6, 128).contiguous()
        self.reg_b6 = f32("dpt_regressor_head.conv2.2.bias")
        # pose head (1x1 convs as GEMMs, MLP tail fp32)
        self.pose_proj, self.pose_proj_b = hlin("pose_head.proj"), f32("pose_head.proj.bias")
        self.pose_res = []
        for b in range(2):
            n = f"pose_head.res_conv.{b}"
            self.pose_res.append([(hlin(f"{n}.res_conv{c}"), f32(f"{n}.res_conv{c}.bias")) for c in (1, 2, 3)])
        self.pose_mlp = [(f32(f"pose_head.more_mlps.{i}.weight"), f32(f"pose_head.more_mlps.{i}.bias")) for i in (0, 2)]
        # fc_t (3) and fc_rot (4) share their input: one 7-row linear gives cat([t, rot]) (pose_head.py:155-158)
        self.pose_tr = (torch.cat([f32("pose_head.fc_t.weight"), f32("pose_head.fc_rot.weight")], 0).contiguous(),
                        torch.cat([f32("pose_head.fc_t.bias"), f32("pose_head.fc_rot.bias")], 0).contiguous())
        self.scale_mlp = [(f32(f"scale_head.{n}.weight"), f32(f"scale_head.{n}.bias"))
                          for n in ("proj", "mlp.0.0", "mlp.1.0", "output_proj")]
        self.norm_mean = torch.tensor(DINOV2_MEAN, device=dev)
        self.norm_std = torch.tensor(DINOV2_STD, device=dev)
        self._geo = None

    def _get(self, name):
        return self.sd[name]

    def geometric(self, sd: Dict[str, object]) -> Dict[str, object]:
        """Kernel-layout weights of the dense (ray, depth) and global (depth-scale, camera) encoders, packed on
        first use.  The reference runs them with autocast disabled (model.py:1377), i.e. as fp32 convs / linears that
        its GPUs run in TF32: fp32 mode keeps fp32 GEMMs; bf16 / fp16 mode runs the dense encoders' convs / linears
        on split operands in the heads' form (head_fmt): TF32-equivalent binary16 [hi | lo] activations against f16
        weights [w | w] (MAPA_F16X2), or the fp32-exact split bf16 (weights [hi | lo | hi] per tap against
        activations read [hi | hi | lo], ~2^-16 relative) with head_precision='fp32' or the bf16 fast-mode heads."""
        if getattr(self, "_geo", None) is not None:
            return self._geo
        dev = self.device
        split = self.lp != torch.float32  # bf16 / fp16 autocast: the encoders' fp32 GEMMs on split operands
        fmt = self.head_fmt if self.head_split else "bf16x3"

        def t(name):
            return torch.from_numpy(np.ascontiguousarray(_np(sd[name]))).to(dev)

        def pack(w):  # [out][taps][cin] fp32 -> fp32 [out][taps*cin], or split-packed ([w | w] f16 / [hi | lo | hi])
            if not split:
                return torch.from_numpy(np.ascontiguousarray(w.reshape(w.shape[0], -1))).to(dev)
            return {"f16": _f16_pack, "f16x2": _f16x2_pack}.get(fmt, _split_pack)(w, dev)

        def c3(name):
            w = _np(sd[f"{name}.weight"])
            return pack(w.transpose(0, 2, 3, 1).reshape(w.shape[0], 9, w.shape[1]))

        def l1(name):
            w = _np(sd[f"{name}.weight"])
            return pack(w.reshape(w.shape[0], 1, -1))

        geo = {}
        for enc in ("ray_dirs_encoder", "depth_encoder"):
            d = dict(conv_in=c3(f"{enc}.conv_in"), conv_in_b=t(f"{enc}.conv_in.bias"), blocks=[],
                     out=l1(f"{enc}.encoder.2"), out_b=t(f"{enc}.encoder.2.bias"),
                     nw=t(f"{enc}.norm_layer.weight"), nb=t(f"{enc}.norm_layer.bias"))
            for i in range(2):
                n = f"{enc}.encoder.{i}"
                d["blocks"].append(dict(c1=c3(f"{n}.conv1"), b1=t(f"{n}.conv1.bias"), c2=c3(f"{n}.conv2"),
                                        b2=t(f"{n}.conv2.bias"), sc=l1(f"{n}.shortcut"), sc_b=t(f"{n}.shortcut.bias")))
            d["split"] = split
            d["fmt"] = fmt
            geo[enc] = d
        for enc in ("depth_scale_encoder", "cam_rot_encoder", "cam_trans_encoder", "cam_trans_scale_encoder"):
            names = ("encoder.0.0.0.0", "encoder.0.0.1", "encoder.0.1", "encoder.1")
            geo[enc] = dict(lin=[(t(f"{enc}.{n}.weight"), t(f"{enc}.{n}.bias")) for n in names],
                            nw=t(f"{enc}.norm_layer.weight"), nb=t(f"{enc}.norm_layer.bias"))
        # lazily built device state is shared by every stream that uses this engine (ranks on threads in the tests,
        # a captured graph's side stream): finish building it before any other stream can read it
        torch.cuda.current_stream(dev).synchronize()
        self._geo = geo
        return geo

    def pos_embed(self, H: int, W: int) -> torch.Tensor:
        """DINOv2 positional embedding for an (H, W) input (vision_transformer.py:208-242).  At 518x518 it is the
        parameter itself; otherwise the reference's bicubic resample of the 37x37 grid, computed once per
        resolution on the host and cached on the device (a parameter transform, not per-inference work)."""
        key = (H, W)
        if key not in self.pos_cache:
            pe = self.pos_embed_param.float()
            h0, w0 = H // PATCH, W // PATCH
            N = pe.shape[1] - 1
            if h0 * w0 == N and H == W:
                out = pe[0]
            else:
                M = int(math.sqrt(N))
                patch = F.interpolate(pe[:, 1:].reshape(1, M, M, ENC_DIM).permute(0, 3, 1, 2), mode="bicubic",
                                      antialias=False, scale_factor=(float(h0 + 0.1) / M, float(w0 + 0.1) / M))
                patch = patch.permute(0, 2, 3, 1).reshape(-1, ENC_DIM)
                out = torch.cat([pe[0, :1], patch], 0)
            out = out.contiguous().to(self.device)
            torch.cuda.current_stream(self.device).synchronize()  # shared lazily built state (see geometric())
            self.pos_cache[key] = out
        return self.pos_cache[key]


def _ceil8(c: int) -> int:
    return (c + 7) // 8 * 8


class MapaEngine:
    def __init__(self, sd: Dict[str, object], device=None, precision: str = "bf16",
                 info: InfoSharingSpec = RELEASED_INFO, heads: str = "fp32"):
        if precision not in ("bf16", "fp16", "fp32"):
            raise ValueError(f"precision must be 'bf16', 'fp16' or 'fp32', got {precision}")
        if heads not in ("tf32", "tf32x2", "fp32", "bf16"):
            raise ValueError(f"heads must be 'tf32' (the reference's GPU recipe), 'tf32x2', 'fp32' (fp32-exact) or "
                             f"'bf16' (fast mode), got {heads}")
        if precision == "fp16" and heads == "bf16":
            raise ValueError("the bf16-heads fast mode is bf16; the fp16 recipe runs the heads at 'tf32' or 'fp32'")
        nat.lib()  # fail loudly without the HIP library / a gfx950 device
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.precision = precision
        # operand dtype of the encoder / transformer GEMMs and attention: bf16 or fp16 autocast (model.py:2287-2302)
        self.lp = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[precision]
        # heads under autocast run as the reference runs them, autocast disabled (model.py:1774), on their own operand
        # form (hsplit): heads='tf32' — the reference's GPU recipe, whose fp32 convs / linears run TF32 (cudnn's
        # default, matmul.allow_tf32 = True at model.py:93): binary16 activations and weights, TF32's 11 significant
        # bits each, fp32 accumulation (MAPA_F16, 1x the bf16 MFMA work); 'tf32x2': binary16 [hi | lo] activations
        # (22 bits) against f16 weights [w | w] (MAPA_F16X2, 2x); 'fp32': fp32-exact split bf16 [hi | lo] read as
        # [hi | hi | lo] against [hi | lo | hi] (MAPA_BF16X3, 3x).  fp32 mode is exact throughout.
        self.heads = "fp32" if precision == "fp32" else heads
        self.hsplit = precision != "fp32" and heads in ("tf32", "tf32x2", "fp32")
        self.hfmt = ({"tf32": "f16", "tf32x2": "f16x2"}.get(heads, "bf16x3")) if self.hsplit else "bf16x3"
        self._sd = sd  # host state dict: the geometric encoders are packed on first use
        self.info = info
        with torch.cuda.device(self.device):
            self.w = PackedWeights(sd, self.device, self.lp, info, head_split=self.hsplit, head_fmt=self.hfmt)

    # ------------------------------------------------------------------------- head operands (model.py:1774)
    def _hop(self, rows, C):
        """Operand buffer of a head GEMM/conv input with C channels: split rows [hi | lo], 2C wide — binary16 for the
        TF32-equivalent heads (read as a plain 2C-wide f16 operand), bf16 for the fp32-exact ones (read as the
        logical K blocks [hi | hi | lo]) — when the heads run split under autocast, else lp rows."""
        if self.hsplit and self.hfmt == "f16":
            return torch.empty(rows, C, dtype=torch.float16, device=self.device)
        if self.hsplit:
            dt = torch.float16 if self.hfmt == "f16x2" else torch.bfloat16
            return torch.empty(rows, 2 * C, dtype=dt, device=self.device)
        return self._empty(rows, C)

    def _hw(self, C):
        """Logical per-pixel K width of a head input with C channels (2C / 3C for the f16x2 / bf16x3 split)."""
        if not self.hsplit or self.hfmt == "f16":
            return C
        return 2 * C if self.hfmt == "f16x2" else 3 * C

    def _hout(self, buf=None, relu=None):
        """GEMM output keywords writing head operands: out_s3 / out_s3_relu in split mode, else out_lp / _relu."""
        d = {}
        s3 = self.hsplit and self.hfmt != "f16"
        if buf is not None:
            d["out_s3" if s3 else "out_lp"] = buf
        if relu is not None:
            d["out_s3_relu" if s3 else "out_lp_relu"] = relu
        return d

    def head_rows(self, x_f32):
        """fp32 rows [R][C] -> a head operand (module-level API inputs, model.py:1774 fp32 heads)."""
        R, C = x_f32.shape
        if self.hsplit and self.hfmt == "f16":
            y = self._hop(R, C)
            nat.convert_rows(x_f32, x_f32.stride(0), R, C, y, C)  # range-checked (MAPA_FAULT_F16_RANGE)
            return y
        if self.hsplit:
            y = self._hop(R, C)
            nat.split_rows(x_f32.contiguous(), R, C, C, y)
            return y
        return x_f32.to(self.lp).contiguous()

    # ---------------------------------------------------------------------------------------- profiling
    def enable_kernel_timing(self):
        nat.timing_start()

    def collect_kernel_timing(self):
        return nat.timing_stop()

    # ----------------------------------------------------------------------------------------------- utils
    def _empty(self, *shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.lp, device=self.device)

    def _const(self, vals, dtype):
        """A small device tensor of host-built values (view indices, per-view masks / scales), cached by value: an
        eager run fills the cache, so a HIP-graph capture of the same structure never copies host memory."""
        key = (tuple(vals) if not isinstance(vals[0], (list, tuple)) else tuple(map(tuple, vals)), dtype)
        cache = self.__dict__.setdefault("_consts", {})
        t = cache.get(key)
        if t is None:
            if torch.cuda.is_current_stream_capturing():
                raise nat.NativeError("geometric-input constants must be built by an eager run before capture")
            t = torch.tensor(vals, dtype=dtype).to(self.device)
            torch.cuda.current_stream(self.device).synchronize()  # shared lazily built state (see geometric())
            cache[key] = t
        return t

    def _ln(self, x, rows, dim, w, b, *, y_f32=None, y_lp=None, y_s3=None, group=0, gstride=0, off=0, ldx=None):
        nat.layernorm(x, rows, dim, w, b, eps=LN_EPS, ldx=ldx, y_f32=y_f32, y_lp=y_lp, y_s3=y_s3, group=group,
                      group_stride=gstride, row_off=off)

    def _ln_head(self, x, rows, dim, w, b, out, **kw):
        """LayerNorm whose output feeds a head: split operand rows in split mode, else lp (or binary16) rows."""
        if self.hsplit and self.hfmt != "f16":
            self._ln(x, rows, dim, w, b, y_s3=out, **kw)
        else:
            self._ln(x, rows, dim, w, b, y_lp=out, **kw)

    def _conv3(self, x, n, IH, IW, C, wmat, Cout, stride=1, **epi):
        OH, OW = (IH + 2 - 3) // stride + 1, (IW + 2 - 3) // stride + 1
        nat.gemm(x, wmat, n * OH * OW, Cout, 9 * C, conv=(C, IH, IW, OH, OW, stride), **epi)
        return OH, OW

    # ------------------------------------------------------------------------------------ transformer block
    def _norm1(self, x, xn, rows, dim, p, normed):
        """norm1 of a block into xn for the rows the previous block's fc2 did not already normalise (normed)."""
        if normed < rows:
            self._ln(x[normed:], rows - normed, dim, p["n1w"], p["n1b"], y_lp=xn[normed:])

    @staticmethod
    def _lnf(w, b, out):
        """The LayerNorm that follows a residual linear, requested from that GEMM (mapa_gemm_desc.ln_*): fused into
        its epilogue where the library can (bf16 residual linears on the 192-row tiles), else run right after it by
        the library with the same kernel as _ln."""
        return dict(ln=(w, b, LN_EPS, out))

    def _block(self, x, xn, qkv, ao, hbuf, rows, dim, heads, p, *, attn_batch, attn_seq, gamma=True,
               attn_kind="attention", attn_scale=None, normed=0, next_ln=None):
        """SelfAttentionBlock / NestedTensorBlock (dinov2 layers/block.py:93-118, transformer_blocks.py:452-469) on the
        fp32 residual stream x.  norm2 comes out of the attention projection's GEMM and, with next_ln = the next
        block's (norm1 weight, bias), that block's norm1 out of fc2's (xn); normed = leading rows of xn already
        holding this block's norm1.  Returns the rows of xn normalised for the next block."""
        self._norm1(x, xn, rows, dim, p, normed)
        nat.gemm(xn, p["qkv"], rows, 3 * dim, dim, bias=p["qkv_b"], out_lp=qkv)
        rs = 3 * dim
        nat.attention(qkv, qkv[:, dim:], qkv[:, 2 * dim:], ao, batch=attn_batch, heads=heads, seq_q=attn_seq,
                      seq_kv=attn_seq, q_bstride=attn_seq * rs, q_rstride=rs, k_bstride=attn_seq * rs, k_rstride=rs,
                      v_bstride=attn_seq * rs, v_rstride=rs, o_bstride=attn_seq * dim, o_rstride=dim, kind=attn_kind,
                      scale=attn_scale)
        nat.gemm(ao, p["proj"], rows, dim, dim, bias=p["proj_b"], gamma=p.get("ls1") if gamma else None,
                 resid1=x, out_f32=x, **self._lnf(p["n2w"], p["n2b"], xn))
        nat.gemm(xn, p["fc1"], rows, 4 * dim, dim, bias=p["fc1_b"], act=nat.ACT_GELU, out_lp=hbuf)
        nat.gemm(hbuf, p["fc2"], rows, dim, 4 * dim, bias=p["fc2_b"], gamma=p.get("ls2") if gamma else None,
                 resid1=x, out_f32=x, **(self._lnf(*next_ln, xn) if next_ln is not None else {}))
        return rows if next_ln is not None else 0

    # ------------------------------------------------------------------------------------------- encoder
    def encode(self, imgs, taps=None, geo: Optional[GeoInputs] = None, scenes: int = 1):
        """DINOv2 ViT-L/14 + final norm [+ geometric-input features] + fusion LayerNorm.  Returns fused_lp
        [VB*T+B][1024] (the last B rows = the B scenes' scale tokens), the same rows in f32 if taps is not None or the
        transformer has no input projection (else None), and the token grid."""
        w = self.w
        B = scenes
        VB, _, H, W = imgs.shape
        hp, wp = H // PATCH, W // PATCH
        T = hp * wp
        enc = self.encoder_features(imgs)
        if taps is not None:
            taps["encoder"] = enc.clone()
        if geo is not None and not geo.empty():
            self.geometric(enc, geo, VB, H, W)
        fused_lp = self._empty(VB * T + B, ENC_DIM)
        identity = w.pe_proj is None  # the transformer reads the fp32 fused rows directly
        need_f32 = taps is not None or identity or self.hsplit  # split heads read the fp32 fused rows (DPT input 0)
        fused_f32 = self._empty(VB * T + B, ENC_DIM, dtype=torch.float32) if need_f32 else None
        self._ln(enc, VB * T, ENC_DIM, w.fus_w, w.fus_b, y_lp=fused_lp, y_f32=fused_f32)
        # the scale token of every scene (source row stride 0: one row replicated)
        nat.convert_rows(w.scale_token.view(1, -1), 0, B, ENC_DIM, fused_lp[VB * T:], ENC_DIM)
        if fused_f32 is not None:
            fused_f32[VB * T:].copy_(w.scale_token.view(1, -1).expand(B, -1))
        if taps is not None:
            taps["fused"] = fused_f32[:VB * T]
        return fused_lp, fused_f32, (hp, wp)

    def encoder_features(self, imgs):
        """DINOv2Encoder.forward (dinov2.py:146-178): patch embed + cls + pos-embed, 24 blocks, final norm.
        Returns the patch-token features [VB*T][1024] f32 (cls dropped)."""
        w = self.w
        VB, _, H, W = imgs.shape
        hp, wp = H // PATCH, W // PATCH
        T = hp * wp
        R = VB * (T + 1)
        patches = self._empty(VB * T, KPAD)
        nat.patchify(imgs, VB, H, W, patches, KPAD)
        pe_out = self._empty(VB * T, ENC_DIM, dtype=torch.float32)
        nat.gemm(patches, w.pe_w, VB * T, ENC_DIM, KPAD, bias=w.pe_b, out_f32=pe_out)
        x = self._empty(R, ENC_DIM, dtype=torch.float32)
        nat.assemble_tokens(pe_out, w.cls, w.pos_embed(H, W), VB, T, ENC_DIM, x)
        del pe_out, patches
        xn, qkv, ao = self._empty(R, ENC_DIM), self._empty(R, 3 * ENC_DIM), self._empty(R, ENC_DIM)
        hbuf = self._empty(R, 4 * ENC_DIM)
        normed = 0
        for i, p in enumerate(w.enc):
            nxt = w.enc[i + 1] if i + 1 < len(w.enc) else None
            normed = self._block(x, xn, qkv, ao, hbuf, R, ENC_DIM, ENC_HEADS, p, attn_batch=VB, attn_seq=T + 1,
                                 normed=normed, next_ln=None if nxt is None else (nxt["n1w"], nxt["n1b"]))
        del xn, qkv, ao, hbuf
        enc = self._empty(VB * T, ENC_DIM, dtype=torch.float32)
        self._ln(x, VB * T, ENC_DIM, w.enc_nw, w.enc_nb, y_f32=enc, group=T, gstride=T + 1, off=1)
        return enc

    # ------------------------------------------------------------------------------ geometric inputs
    def geometric(self, enc, geo: GeoInputs, VB, H, W):
        """enc [VB*T][1024] f32 += ray / depth dense features and the per-view global features, in the reference's
        order (model.py:1392-1420): rays, depth (+ depth scale), camera rotation, translation, translation scale.
        fp32 kernels throughout (autocast disabled in the reference, model.py:1377)."""
        g = self.w.geometric(self._sd)
        T = (H // PATCH) * (W // PATCH)
        f32 = torch.float32
        dev = self.device
        if geo.ray_views:
            self._dense_into(enc, geo.rays, geo.ray_views, VB, H, W, 3, g["ray_dirs_encoder"])
        vecs, scales = [], []
        if geo.depth_views:
            nf = self._empty(VB, dtype=f32)
            log_nf = self._empty(VB, dtype=f32)
            nat.depth_norm_factors(geo.depth, VB, H * W, nf, log_nf)
            self._dense_into(enc, geo.depth, geo.depth_views, VB, H, W, 1, g["depth_encoder"], view_div=nf)
            sel = set(geo.depth_views)
            sc = [1.0 if (v in sel and geo.depth_metric[v]) else 0.0 for v in range(VB)]
            if any(sc):
                vecs.append(self._global_rep(log_nf.view(VB, 1), VB, 1, g["depth_scale_encoder"]))
                scales.append(sc)
        if any(geo.cam_mask):
            NV = len(geo.cam_mask)  # all views (of every scene)
            V = NV // geo.scenes
            mask = self._const([1 if m else 0 for m in geo.cam_mask], torch.uint8)
            q = self._empty(NV, 4, dtype=f32)
            t = self._empty(NV, 3, dtype=f32)
            lnf = self._empty(NV, dtype=f32)
            cq, ct = geo.cam_quats.contiguous(), geo.cam_trans.contiguous()
            for b in range(geo.scenes):  # camera inputs in each scene's view-0 frame, translations normalised per scene
                sl = slice(b * V, (b + 1) * V)
                nat.pose_inputs(cq[sl], ct[sl], mask[sl], V, q[sl], t[sl], lnf[sl])
            # this rank's images among all views: scene b's local view i (image b*c + i) is view b*V + s0 + i
            s0, c = geo.local_start, VB // geo.scenes
            loc = [b * V + s0 + i for b in range(geo.scenes) for i in range(c)]
            if loc == list(range(s0, s0 + VB)):  # one contiguous run (one scene, or B scenes unsharded)
                pick = lambda a: a[s0:s0 + VB]  # noqa: E731
            else:  # B scenes on a view shard
                li = self._const(loc, torch.long)
                pick = lambda a: a.index_select(0, li)  # noqa: E731
            cm = [1.0 if geo.cam_mask[j] else 0.0 for j in loc]
            pm = [cm[v] if geo.pose_metric[j] else 0.0 for v, j in enumerate(loc)]
            vecs.append(self._global_rep(pick(q), VB, 4, g["cam_rot_encoder"]))
            scales.append(cm)
            vecs.append(self._global_rep(pick(t), VB, 3, g["cam_trans_encoder"]))
            scales.append(cm)
            if any(pm):
                vecs.append(self._global_rep(pick(lnf).view(VB, 1), VB, 1, g["cam_trans_scale_encoder"]))
                scales.append(pm)
        if vecs:
            vb = torch.stack(vecs, 0).contiguous()
            sb = self._const(scales, f32)
            nat.add_view_vectors(enc, T, ENC_DIM, VB, vb, sb, len(vecs))

    def _dense_into(self, enc, data, views, VB, H, W, C, g, view_div=None):
        """DenseRepresentationEncoder (dense_rep_encoder.py:234-287, apply_pe=False) on the selected local views,
        added into their encoder rows (features * mask, model.py:960-968 / 1136-1140)."""
        hp, wp = H // PATCH, W // PATCH
        T = hp * wp
        n = len(views)
        if n != VB:
            idx = self._const(list(views), torch.long)
            data = data.index_select(0, idx)
            if view_div is not None:
                view_div = view_div.index_select(0, idx)
        data = data.contiguous()
        f = self._dense_rep(data, n, H, W, C, g, view_div)
        runs = []
        for i, v in enumerate(views):
            if runs and runs[-1][1] + runs[-1][2] == v:
                runs[-1][2] += 1
            else:
                runs.append([i, v, 1])
        for i, v, k in runs:
            nat.add_f32(enc[v * T:(v + k) * T], f[i * T:(i + k) * T], k * T * ENC_DIM)

    def _dense_rep(self, data, n, H, W, C, g, view_div=None):
        f32 = torch.float32
        hp, wp = H // PATCH, W // PATCH
        M = n * hp * wp
        cin = C * PATCH * PATCH

        def operand(x, c):  # GEMM A operand and its logical per-tap width: fp32 as is, or split [hi | lo]
            if not g["split"]:
                return x, c
            cp = _ceil8(c)
            if g.get("fmt") == "f16":  # binary16 rows, zero-padded to cp
                y = self._empty(M, cp, dtype=torch.float16)
                if cp != c:
                    y[:, c:].zero_()
                nat.convert_rows(x, c, M, c, y, cp)
                return y, cp
            f16 = g.get("fmt") == "f16x2"
            y = self._empty(M, 2 * cp, dtype=torch.float16 if f16 else torch.bfloat16)
            nat.split_rows(x, M, c, cp, y)
            return y, (2 if f16 else 3) * cp

        u = self._empty(M, cin, dtype=f32)
        nat.pixel_unshuffle(data, n, H, W, C, PATCH, u, view_div=view_div)
        c0 = g["conv_in"].shape[0]
        x = self._empty(M, c0, dtype=f32)
        a, k = operand(u, cin)
        del u
        nat.gemm(a, g["conv_in"], M, c0, 9 * k, bias=g["conv_in_b"], out_f32=x, conv=(k, hp, wp, hp, wp, 1))
        del a
        cin = c0
        for blk in g["blocks"]:
            co = blk["c1"].shape[0]
            a, k = operand(x, cin)
            idt = self._empty(M, co, dtype=f32)
            nat.gemm(a, blk["sc"], M, co, k, bias=blk["sc_b"], out_f32=idt)
            o = self._empty(M, co, dtype=f32)
            nat.gemm(a, blk["c1"], M, co, 9 * k, bias=blk["b1"], act=nat.ACT_GELU, out_f32=o,
                     conv=(k, hp, wp, hp, wp, 1))
            del a
            a, k = operand(o, co)
            del o
            x = self._empty(M, co, dtype=f32)
            nat.gemm(a, blk["c2"], M, co, 9 * k, bias=blk["b2"], resid1=idt, act=nat.ACT_GELU_POST, out_f32=x,
                     conv=(k, hp, wp, hp, wp, 1))
            del idt, a
            cin = co
        y = self._empty(M, ENC_DIM, dtype=f32)
        a, k = operand(x, cin)
        del x
        nat.gemm(a, g["out"], M, ENC_DIM, k, bias=g["out_b"], out_f32=y)
        del a
        f = self._empty(M, ENC_DIM, dtype=f32)
        nat.layernorm(y, M, ENC_DIM, g["nw"], g["nb"], eps=LN_EPS, y_f32=f)
        return f

    def _global_rep(self, inp, m, cin, g):
        """GlobalRepresentationEncoder (global_rep_encoder.py:85-104): 3x (Linear + GELU), Linear, LayerNorm."""
        f32 = torch.float32
        inp = inp.contiguous()
        h = inp
        k = cin
        for i, (w_, b_) in enumerate(g["lin"]):
            n_out = w_.shape[0]
            o = self._empty(m, n_out, dtype=f32)
            nat.linear_small(h, m, k, w_, b_, n_out, nat.ACT_GELU if i < 3 else nat.ACT_NONE, o)
            h, k = o, n_out
        y = self._empty(m, ENC_DIM, dtype=f32)
        nat.layernorm(h, m, ENC_DIM, g["nw"], g["nb"], eps=LN_EPS, y_f32=y)
        return y

    # ----------------------------------------------------------------------------------------------- AAT
    def aat(self, fused_lp, VB, T, taps=None, shard=None, comm=None, pe_idx=None, fused_f32=None, scenes: int = 1):
        """The multi-view transformer with intermediate-feature return: AAT (alternating_attention_transformer.py:
        530-771; released config: 24 blocks, taps after 11 and 17) or GAT (global_attention_transformer.py:458-640:
        every block global), per self.info.  Returns the list of normed taps (2 or 3, VB*T rows) and the final
        features as head operands (_hop: split rows or lp), and the final scale-token feature (f32, dim).  fused_f32: the fp32 fused rows (with the scale token), needed
        when proj_embed is the identity.  pe_idx: (V_total,) int64 device tensor of view-PE table rows (row 0 for the
        reference view) when the variant encodes non-reference views too.  With `shard` (parallel.ShardPlan) this
        rank holds only its views (+ the scale-token replica) and the global layers all-gather K/V through `comm`.
        scenes = B > 1: VB = B x V images scene-major, rows [image][token] then the B scale tokens; frame layers run
        over all images at once, global layers attend within each scene (its tokens + its scale token).  With a shard
        too, V is this rank's view count of every scene (ShardPlan.scenes = B)."""
        w, info = self.w, self.info
        D, NH = info.dim, info.heads
        B = scenes
        if B > 1 and (taps is not None or VB % B or (shard is not None and shard.scenes != B)):
            raise ValueError("batched scenes: no taps, VB a multiple of the scene count, a shard plan of B scenes")
        V = VB // B
        L = VB * T + B
        if w.pe_proj is None:  # identity projection: the residual stream starts from the fp32 fused features
            if fused_f32 is None:
                raise ValueError("this info-sharing variant has no input projection: pass fused_f32")
            y = fused_f32.clone() if taps is not None else fused_f32
        else:
            y = self._empty(L, D, dtype=torch.float32)
            nat.gemm(fused_lp, w.pe_proj, L, D, ENC_DIM, bias=w.pe_proj_b, out_f32=y)
        first = 0 if shard is None else shard.starts[shard.rank]  # global index of this rank's first view
        if info.nonref_pe:  # view PE on every view: table rows pe_idx (row 0 on the reference view); one draw for
            # all scenes, as the reference's forward draws once and repeats it over the batch
            vecs = w.view_pos.index_select(0, pe_idx[first:first + V]).repeat(B, 1).contiguous()
            nat.add_view_vectors(y, T, D, VB, vecs, self._ones(VB), 1)
        elif info.ref_pe and first == 0:  # reference-view PE on view 0 (of every scene) only
            for b in range(B):
                nat.add_rowvec(y, D, b * V * T, b * V * T + T, D, w.view_pe)
        yn, qkv, ao = self._empty(L, D), self._empty(L, 3 * D), self._empty(L, D)
        hbuf = self._empty(L, 4 * D)
        # tokens one global block attends to (a scene's views + its scale token)
        L_all = V * T + 1 if shard is None else shard.total_kv
        g_scale = 0.125 * info.q_scale(L_all) if (info.scalable_softmax or info.entropy_scaling) else None
        f_scale = 0.125 * info.q_scale(T) if (info.scalable_softmax or info.entropy_scaling) else None
        if shard is not None:
            kv_full = self._empty(shard.world * shard.max_rows, 2 * D)
            q_loc = self._empty(L, D)
        inter = {}
        normed = 0  # leading rows of yn already holding the current block's norm1 (fused into the last fc2)
        for d, p in enumerate(w.aat):
            nxt = w.aat[d + 1] if d + 1 < len(w.aat) else None
            nln = None if nxt is None else (nxt["n1w"], nxt["n1b"])
            if info.is_global(d):   # global attention over every view + the scale token
                if shard is None and B == 1:
                    normed = self._block(y, yn, qkv, ao, hbuf, L, D, NH, p, attn_batch=1, attn_seq=L, gamma=False,
                                         attn_kind="attention_global", attn_scale=g_scale, normed=normed,
                                         next_ln=nln)
                elif shard is None:
                    normed = self._block_global_scenes(y, yn, qkv, ao, hbuf, L, p, B, V, T, g_scale, normed, nln)
                elif B == 1:
                    normed = self._block_global_sharded(y, yn, q_loc, kv_full, ao, hbuf, L, p, shard, comm, g_scale,
                                                        normed, nln)
                else:
                    normed = self._block_global_sharded_scenes(y, yn, q_loc, kv_full, ao, hbuf, L, p, shard, comm,
                                                               V, T, g_scale, normed, nln)
            else:                   # frame attention inside each view; the scale token bypasses the block
                normed = self._block(y, yn, qkv, ao, hbuf, VB * T, D, NH, p, attn_batch=VB, attn_seq=T,
                                     gamma=False, attn_scale=f_scale, normed=normed, next_ln=nln)
            if d in info.indices:  # IFR taps feed only the DPT (a head: fp32 in the reference, model.py:1774)
                t_lp = self._hop(VB * T, D)
                t_f = self._empty(VB * T, D, dtype=torch.float32) if taps is not None else None
                self._ln_head(y, VB * T, D, w.aat_nw, w.aat_nb, t_lp, y_f32=t_f)
                inter[d] = t_lp
                if taps is not None:
                    taps[f"aat_l{d}"] = t_f
                    tk = self._empty(1, D, dtype=torch.float32)  # the scale token, normed as well
                    self._ln(y[VB * T:], 1, D, w.aat_nw, w.aat_nb, y_f32=tk)
                    taps[f"aat_l{d}_token"] = tk
        del yn, qkv, ao, hbuf
        fin_lp = self._hop(L, D)  # the final features feed the DPT and the pose head only
        fin_f32 = self._empty(L, D, dtype=torch.float32)
        self._ln_head(y, L, D, w.aat_nw, w.aat_nb, fin_lp, y_f32=fin_f32)
        if shard is not None and (shard.world > 1 or force_collectives()):
            # the scale-token replicas round differently per rank (query blocking, merge order): rank 0's final
            # scale-token feature is the one every rank's scale head reads (one D-float broadcast)
            comm.broadcast_(fin_f32[VB * T:], 0)
        if taps is not None:
            taps["aat_final"] = fin_f32[:VB * T]
            taps["scale_token"] = fin_f32[VB * T]
        return [inter[i] for i in info.indices], fin_lp, fin_f32[VB * T:]

    def _ones(self, n):
        o = getattr(self, "_ones_buf", None)
        if o is None or o.numel() < n:
            o = torch.ones(max(n, 64), dtype=torch.float32, device=self.device)
            torch.cuda.current_stream(self.device).synchronize()  # shared lazily built state (see geometric())
            self._ones_buf = o
        return o

    def _block_global_scenes(self, y, yn, qkv, ao, hbuf, L, p, B, V, T, scale=None, normed=0, next_ln=None):
        """Global SelfAttentionBlock of B batched scenes (rows [image][token] scene-major, then the B scale tokens):
        LayerNorm / GEMMs over all rows at once; per scene one attention of its token rows and one of its scale-token
        row, both over the scene's keys through the segment table (its V*T token rows + its scale-token row)."""
        C, NH = self.info.dim, self.info.heads
        rs = 3 * C
        self._norm1(y, yn, L, C, p, normed)
        nat.gemm(yn, p["qkv"], L, rs, C, bias=p["qkv_b"], out_lp=qkv)
        k, v = qkv[:, C:], qkv[:, 2 * C:]
        kw = dict(batch=1, heads=NH, q_bstride=0, q_rstride=rs, k_bstride=0, k_rstride=rs, v_bstride=0, v_rstride=rs,
                  o_bstride=0, o_rstride=C, scale=scale, kind="attention_global")
        for b in range(B):
            r0, tok = b * V * T, V * T * B + b
            segs = [(r0, V * T), (tok, 1)]
            nat.attention(qkv[r0:], k, v, ao[r0:], seq_q=V * T, seq_kv=V * T + 1, kv_segments=segs, **kw)
            nat.attention(qkv[tok:], k, v, ao[tok:], seq_q=1, seq_kv=V * T + 1, kv_segments=segs, **kw)
        nat.gemm(ao, p["proj"], L, C, C, bias=p["proj_b"], resid1=y, out_f32=y, **self._lnf(p["n2w"], p["n2b"], yn))
        nat.gemm(yn, p["fc1"], L, 4 * C, C, bias=p["fc1_b"], act=nat.ACT_GELU, out_lp=hbuf)
        nat.gemm(hbuf, p["fc2"], L, C, 4 * C, bias=p["fc2_b"], resid1=y, out_f32=y,
                 **(self._lnf(*next_ln, yn) if next_ln is not None else {}))
        return L if next_ln is not None else 0

    def _block_global_sharded(self, y, yn, q_loc, kv_full, ao, hbuf, L, p, shard, comm, scale=None, normed=0,
                              next_ln=None):
        """Global SelfAttentionBlock on a view shard: Q for the local rows, K/V of all ranks (one all-gather).
        The all-gather runs on the communicator's stream while the local queries attend to this rank's own keys;
        the remote-key partial follows the gather and the two partials are merged through their LSEs
        (MAPA_KV_OVERLAP=0: gather first, one attention over every key)."""
        C, NH = self.info.dim, self.info.heads
        self._norm1(y, yn, L, C, p, normed)
        nat.gemm(yn, p["qkv"][:C], L, C, C, bias=p["qkv_b"][:C], out_lp=q_loc)
        slot = kv_full[shard.rank * shard.max_rows:]
        nat.gemm(yn, p["qkv"][C:], L, 2 * C, C, bias=p["qkv_b"][C:], out_lp=slot, ldo=2 * C)
        strides = dict(batch=1, heads=NH, seq_q=L, q_bstride=0, q_rstride=C, k_bstride=0, k_rstride=2 * C,
                       v_bstride=0, v_rstride=2 * C, o_bstride=0, o_rstride=C, scale=scale)
        overlap = hasattr(comm, "allgather_slots_async") and os.environ.get("MAPA_KV_OVERLAP", "1") != "0"
        # MAPA_FORCE_OVERLAP=1 on a one-rank shard: the overlapped multi-rank branch with the second half of this
        # rank's own keys standing in for the remote ones (parallel.force_overlap)
        split_own = shard.world == 1 and overlap and force_overlap()
        if shard.world == 1 and not force_collectives():  # a one-rank group: every key is local
            nat.attention(q_loc, kv_full, kv_full[:, C:], ao, seq_kv=shard.total_kv,
                          kv_segments=shard.kv_segments(), kind="attention_global", **strides)
        elif not overlap or (shard.world == 1 and not split_own):  # gather first (forced collectives, one rank)
            comm.allgather_slots(kv_full, shard.max_rows)
            nat.attention(q_loc, kv_full, kv_full[:, C:], ao, seq_kv=shard.total_kv,
                          kv_segments=shard.kv_segments(), kind="attention_global", **strides)
        else:
            handle = comm.allgather_slots_async(kv_full, shard.max_rows)
            segs = shard.kv_segments()
            if split_own:
                st, n = segs[0]
                own, rest = (st, n // 2), [(st + n // 2, n - n // 2)]
            else:
                own = segs[shard.rank]
                rest = [sg for r, sg in enumerate(segs) if r != shard.rank]
            lse_l = self._empty(NH, L, dtype=torch.float32)
            # eager timing pass (bench.py kv_overlap): local- and remote-key attention and the join's exposed wait on
            # this stream; the all-gather itself is timed on the communicator's stream (RcclComm)
            t0 = nat.mark()
            nat.attention(q_loc, kv_full, kv_full[:, C:], ao, seq_kv=own[1], kv_segments=[own], lse=lse_l,
                          kind="attention_global", **strides)
            t1 = nat.mark()
            handle.wait()
            t2 = nat.mark()
            ao_r = self._empty(L, C)
            lse_r = self._empty(NH, L, dtype=torch.float32)
            nat.attention(q_loc, kv_full, kv_full[:, C:], ao_r, seq_kv=sum(sg[1] for sg in rest), kv_segments=rest,
                          lse=lse_r, kind="attention_global", **strides)
            t3 = nat.mark()
            nat.span("kv_local_attention", t0, t1)
            nat.span("kv_gather_wait", t1, t2)
            nat.span("kv_remote_attention", t2, t3)
            nat.attn_merge(ao, lse_l, ao_r, lse_r, ao, L, NH, C)
        nat.gemm(ao, p["proj"], L, C, C, bias=p["proj_b"], resid1=y, out_f32=y, **self._lnf(p["n2w"], p["n2b"], yn))
        nat.gemm(yn, p["fc1"], L, 4 * C, C, bias=p["fc1_b"], act=nat.ACT_GELU, out_lp=hbuf)
        nat.gemm(hbuf, p["fc2"], L, C, 4 * C, bias=p["fc2_b"], resid1=y, out_f32=y,
                 **(self._lnf(*next_ln, yn) if next_ln is not None else {}))
        return L if next_ln is not None else 0

    def _block_global_sharded_scenes(self, y, yn, q_loc, kv_full, ao, hbuf, L, p, shard, comm, V, T, scale=None,
                                     normed=0, next_ln=None):
        """Global SelfAttentionBlock of B batched scenes on a view shard (V = this rank's views per scene): Q for the
        local rows, K/V of every rank in one slot all-gather, then per scene one attention of its local token rows
        and one of its scale-token replica, both over the scene's keys on every rank (ShardPlan.scene_kv_segments).
        The gather runs before the attention (the B = 1 layer overlaps it with the own-key partial)."""
        C, NH = self.info.dim, self.info.heads
        B = shard.scenes
        self._norm1(y, yn, L, C, p, normed)
        nat.gemm(yn, p["qkv"][:C], L, C, C, bias=p["qkv_b"][:C], out_lp=q_loc)
        slot = kv_full[shard.rank * shard.max_rows:]
        nat.gemm(yn, p["qkv"][C:], L, 2 * C, C, bias=p["qkv_b"][C:], out_lp=slot, ldo=2 * C)
        if shard.world > 1 or force_collectives():
            comm.allgather_slots(kv_full, shard.max_rows)
        kw = dict(batch=1, heads=NH, q_bstride=0, q_rstride=C, k_bstride=0, k_rstride=2 * C, v_bstride=0,
                  v_rstride=2 * C, o_bstride=0, o_rstride=C, scale=scale, kind="attention_global")
        k, v = kv_full, kv_full[:, C:]
        for b in range(B):
            r0, tok = b * V * T, V * T * B + b
            segs = shard.scene_kv_segments(b)
            nat.attention(q_loc[r0:], k, v, ao[r0:], seq_q=V * T, seq_kv=shard.total_kv, kv_segments=segs, **kw)
            nat.attention(q_loc[tok:], k, v, ao[tok:], seq_q=1, seq_kv=shard.total_kv, kv_segments=segs, **kw)
        nat.gemm(ao, p["proj"], L, C, C, bias=p["proj_b"], resid1=y, out_f32=y, **self._lnf(p["n2w"], p["n2b"], yn))
        nat.gemm(yn, p["fc1"], L, 4 * C, C, bias=p["fc1_b"], act=nat.ACT_GELU, out_lp=hbuf)
        nat.gemm(hbuf, p["fc2"], L, C, 4 * C, bias=p["fc2_b"], resid1=y, out_f32=y,
                 **(self._lnf(*next_ln, yn) if next_ln is not None else {}))
        return L if next_ln is not None else 0

    # ----------------------------------------------------------------------------------------------- DPT
    def dpt(self, fused_lp, l11, l17, fin_lp, VB, hp, wp, H, W, taps=None, head=None, join=None):
        """DPTFeature + DPTRegressionProcessor (dpt.py:180-311).  Inputs are head operands (_hop rows); fused_lp
        is the first DPT input — the fused encoder features (ENC_DIM) or, with three info-sharing taps
        (model.py:1748-1768), the first tap; its width comes from the packed weight.  Returns the ReLU'd 128-ch
        hidden map at HxW (fp32 in split mode, else lp), or None when `head` (see dpt_regress) took the dense head
        into the last conv.  join: called right before the first kernel that reads `head`'s pose / scale rows (the
        pose / scale heads' branch, run_heads)."""
        owned = [self.dpt_feature(fused_lp, l11, l17, fin_lp, VB, hp, wp, taps)[0]]
        return self.dpt_regress(owned, VB, 8 * hp, 8 * wp, H, W, head, join)  # freed after its first conv

    def fused_head_out(self):
        """Whether the regressor's conv2 can carry the dense head in its epilogue (mapa_regressor_head_out: bf16 or
        f16 operands, channel-block-major conv weight).  MAPA_FUSED_HEAD=0 keeps the two launches (A/B)."""
        c2 = self.w.reg_c2
        return (c2.dtype in (torch.bfloat16, torch.float16) and getattr(c2, "_mapa_kblock", 0) == 32
                and os.environ.get("MAPA_FUSED_HEAD", "1") != "0")

    def _hconv3(self, x, n, IH, IW, C, wmat, Cout, stride=1, **epi):
        """3x3 conv of a head operand with C logical channels."""
        return self._conv3(x, n, IH, IW, self._hw(C), wmat, Cout, stride=stride, **epi)

    def _hmap(self, rows, C):
        """A head feature map that is re-read by a bilinear resize: fp32 in split mode, else lp."""
        return self._empty(rows, C, dtype=torch.float32 if self.hsplit else self.lp)

    def dpt_feature(self, fused_lp, l11, l17, fin_lp, VB, hp, wp, taps=None, want_f32=False):
        """DPTFeature (dpt.py:180-232): the four IFR features [VB*T][C] (head operands) -> the 256-ch map at 8x
        [VB][8hp][8wp][256] (head operand; f32 copy too if taps is given or want_f32)."""
        w = self.w
        n, T = VB, hp * wp
        D = self.info.dim
        # input_process 0: 1x1 1024 (or 768)->96, ConvT k4 s4, layer1_rn 3x3 96->256 (no bias)
        a = self._hop(n * T, 96)
        nat.gemm(fused_lp, w.ip[0]["w"], n * T, 96, w.ip[0]["w"].shape[1], bias=w.ip[0]["b"], **self._hout(a))
        up0 = self._hop(n * 16 * T, 96)
        nat.gemm(a, w.ip[0]["ct"], n * T, 16 * 96, self._hw(96), bias=w.ip[0]["ct_b"], bias_mod=96,
                 pixshuf=(4, hp, wp, 96), **self._hout(up0))
        h0, w0 = 4 * hp, 4 * wp
        L0f = self._empty(n * h0 * w0, 256, dtype=torch.float32)
        L0r = self._hop(n * h0 * w0, 256)
        self._hconv3(up0, n, h0, w0, 96, w.layer_rn[0], 256, out_f32=L0f, **self._hout(relu=L0r))
        del a, up0
        # input_process 1: 1x1 768->192, ConvT k2 s2, layer2_rn
        a = self._hop(n * T, 192)
        nat.gemm(l11, w.ip[1]["w"], n * T, 192, self._hw(D), bias=w.ip[1]["b"], **self._hout(a))
        up1 = self._hop(n * 4 * T, 192)
        nat.gemm(a, w.ip[1]["ct"], n * T, 4 * 192, self._hw(192), bias=w.ip[1]["ct_b"], bias_mod=192,
                 pixshuf=(2, hp, wp, 192), **self._hout(up1))
        h1, w1 = 2 * hp, 2 * wp
        L1f = self._empty(n * h1 * w1, 256, dtype=torch.float32)
        L1r = self._hop(n * h1 * w1, 256)
        self._hconv3(up1, n, h1, w1, 192, w.layer_rn[1], 256, out_f32=L1f, **self._hout(relu=L1r))
        del a, up1
        # input_process 2: 1x1 768->384, layer3_rn
        a = self._hop(n * T, 384)
        nat.gemm(l17, w.ip[2]["w"], n * T, 384, self._hw(D), bias=w.ip[2]["b"], **self._hout(a))
        L2f = self._empty(n * T, 256, dtype=torch.float32)
        L2r = self._hop(n * T, 256)
        self._hconv3(a, n, hp, wp, 384, w.layer_rn[2], 256, out_f32=L2f, **self._hout(relu=L2r))
        del a
        # input_process 3: 1x1 768->768, 3x3 s2 768->768, layer4_rn
        a = self._hop(n * T, 768)
        nat.gemm(fin_lp, w.ip[3]["w"], n * T, 768, self._hw(D), bias=w.ip[3]["b"], **self._hout(a))
        h3, w3 = (hp - 1) // 2 + 1, (wp - 1) // 2 + 1
        b3 = self._hop(n * h3 * w3, 768)
        self._hconv3(a, n, hp, wp, 768, w.ip[3]["c3"], 768, stride=2, bias=w.ip[3]["c3_b"], **self._hout(b3))
        L3f = self._empty(n * h3 * w3, 256, dtype=torch.float32)
        L3r = self._hop(n * h3 * w3, 256)
        self._hconv3(b3, n, h3, w3, 768, w.layer_rn[3], 256, out_f32=L3f, **self._hout(relu=L3r))
        del a, b3
        # refinenet4 (RCU2 only) -> x2 -> crop to (hp, wp) -> out_conv
        o = self._fusion_single(n, h3, w3, 4, L3f, L3r)
        path = self._upsample_outconv(o, n, h3, w3, 4, crop=(hp, wp))
        # refinenet3/2/1
        o = self._fusion_two(n, hp, wp, 3, path, L2f, L2r)
        path = self._upsample_outconv(o, n, hp, wp, 3)
        o = self._fusion_two(n, h1, w1, 2, path, L1f, L1r)
        path = self._upsample_outconv(o, n, h1, w1, 2)
        o = self._fusion_two(n, h0, w0, 1, path, L0f, L0r)
        t = taps if taps is not None else ({} if want_f32 else None)
        feat_lp = self._upsample_outconv(o, n, h0, w0, 1, lowp=True, taps=t)
        return feat_lp, (t["dpt_feature"] if t is not None else None)

    def dpt_regress(self, feat_lp, n, hf, wf, H, W, head=None, join=None):
        """DPTRegressionProcessor up to the last ReLU (dpt.py:285-311): conv3x3 256->128 at 8x, bilinear
        (align_corners) to HxW, conv3x3 128->128 + ReLU -> hidden [n*H*W][128] (fp32 in split mode, else lp).
        feat_lp (a head operand) may be a one-element list, handed over so that the 8x map is freed as soon as it
        has been read.  head = (pose_out rows, scale, pts3d, pts3d_cam, rays, depth, conf, logits, mask) of these
        views: the conv's epilogue runs the 1x1 conv 128->6 and the dense head instead (nat.gemm head_out, the
        hidden map never reaches HBM); returns None then."""
        w = self.w
        if isinstance(feat_lp, list):
            feat_lp = feat_lp.pop()
        r1 = self._hmap(n * hf * wf, 128)
        self._hconv3(feat_lp, n, hf, wf, 256, w.reg_c1, 128, bias=w.reg_b1,
                     **({"out_f32": r1} if self.hsplit else {"out_lp": r1}))
        del feat_lp
        r1u = self._hop(n * H * W, 128)
        nat.bilinear_ac(r1, n, hf, wf, 128, H, W, H, W, r1u, split_out=self.hsplit and self.hfmt != "f16")
        del r1
        if head is not None:
            if join is not None:
                join()
            self._hconv3(r1u, n, H, W, 128, w.reg_c2, 128, bias=w.reg_b2, act=nat.ACT_RELU,
                         head_out=(w.reg_w6, w.reg_b6) + tuple(head))
            return None
        hid = self._hmap(n * H * W, 128)
        self._hconv3(r1u, n, H, W, 128, w.reg_c2, 128, bias=w.reg_b2, act=nat.ACT_RELU,
                     **({"out_f32": hid} if self.hsplit else {"out_lp": hid}))
        return hid

    def _fusion_single(self, n, h, w_, r, x_f, x_r):
        u = self.w.refine[r]["resConfUnit2"]
        c1 = self._hop(n * h * w_, 256)
        self._hconv3(x_r, n, h, w_, 256, u["c1"], 256, bias=u["b1"], act=nat.ACT_RELU, **self._hout(c1))
        o = self._hop(n * h * w_, 256)  # out_conv's operand (_upsample_outconv)
        self._hconv3(c1, n, h, w_, 256, u["c2"], 256, bias=u["b2"], resid1=x_f, **self._hout(o))
        return o

    def _fusion_two(self, n, h, w_, r, path_f, skip_f, skip_r):
        d = self.w.refine[r]
        u = d["resConfUnit1"]
        c1 = self._hop(n * h * w_, 256)
        self._hconv3(skip_r, n, h, w_, 256, u["c1"], 256, bias=u["b1"], act=nat.ACT_RELU, **self._hout(c1))
        s_f = self._empty(n * h * w_, 256, dtype=torch.float32)
        s_r = self._hop(n * h * w_, 256)
        self._hconv3(c1, n, h, w_, 256, u["c2"], 256, bias=u["b2"], resid1=skip_f, resid2=path_f, out_f32=s_f,
                     **self._hout(relu=s_r))
        u = d["resConfUnit2"]
        self._hconv3(s_r, n, h, w_, 256, u["c1"], 256, bias=u["b1"], act=nat.ACT_RELU, **self._hout(c1))
        o = self._hop(n * h * w_, 256)
        self._hconv3(c1, n, h, w_, 256, u["c2"], 256, bias=u["b2"], resid1=s_f, **self._hout(o))
        return o

    def _upsample_outconv(self, o, n, h, w_, r, crop=None, lowp=False, taps=None):
        """The fusion block's tail (dpt_block.py:242-254, dpt.py:213): bilinear x2 (align_corners) [+ crop], then the
        1x1 out_conv.  Run here in the other order — out_conv on the h x w map, then the resize of its fp32 output:
        a 1x1 conv mixes channels per pixel and the resize mixes pixels per channel with weights that sum to one, so
        the two commute (bias included; the crop too) up to fp32 rounding, and the GEMM does a quarter of the
        reference's work.  o: the operand rows [n*h*w] (head operand); returns the fp32 map at 2h x 2w (cropped),
        or with lowp a head operand (+ the fp32 tap)."""
        d = self.w.refine[r]
        Hf, Wf = 2 * h, 2 * w_
        oh, ow = crop if crop is not None else (Hf, Wf)
        y = self._empty(n * h * w_, 256, dtype=torch.float32)
        nat.gemm(o, d["out"], n * h * w_, 256, self._hw(256), bias=d["out_b"], out_f32=y)
        if lowp:
            out = self._hop(n * oh * ow, 256)
            nat.bilinear_ac(y, n, h, w_, 256, Hf, Wf, oh, ow, out, split_out=self.hsplit and self.hfmt != "f16")
            if taps is not None:
                f = self._empty(n * oh * ow, 256, dtype=torch.float32)
                nat.bilinear_ac(y, n, h, w_, 256, Hf, Wf, oh, ow, f)
                taps["dpt_feature"] = f.view(n, oh, ow, 256)
            return out
        out = self._empty(n * oh * ow, 256, dtype=torch.float32)
        nat.bilinear_ac(y, n, h, w_, 256, Hf, Wf, oh, ow, out)
        return out

    # ------------------------------------------------------------------------------------- pose / scale
    def _head_stream(self):
        """The side stream of the pose / scale heads' branch (run_heads), one per engine; None runs them in line
        (MAPA_HEAD_BRANCH=0, A/B)."""
        if os.environ.get("MAPA_HEAD_BRANCH", "1") == "0":
            return None
        st = self.__dict__.get("_side_stream")
        if st is None:
            st = self._side_stream = torch.cuda.Stream(self.device)
        return st

    def pose(self, fin_lp, VB, T, taps=None):
        """PoseHead (pose_head.py:50-159) on the final features (a head operand) -> raw (VB, 7)."""
        w = self.w
        M = VB * T
        pf = self._empty(M, POSE_DIM, dtype=torch.float32)
        pl = self._hop(M, POSE_DIM)
        nat.gemm(fin_lp, w.pose_proj, M, POSE_DIM, self._hw(self.info.dim), bias=w.pose_proj_b, out_f32=pf,
                 **self._hout(pl))
        t1, t2 = self._hop(M, POSE_DIM), self._hop(M, POSE_DIM)
        K = self._hw(POSE_DIM)
        for blk in w.pose_res:
            (w1, b1), (w2, b2), (w3, b3) = blk
            nat.gemm(pl, w1, M, POSE_DIM, K, bias=b1, act=nat.ACT_RELU, **self._hout(t1))
            nat.gemm(t1, w2, M, POSE_DIM, K, bias=b2, act=nat.ACT_RELU, **self._hout(t2))
            nat.gemm(t2, w3, M, POSE_DIM, K, bias=b3, act=nat.ACT_RELU, resid1=pf, out_f32=pf, **self._hout(pl))
        pooled = self._empty(VB, POSE_DIM, dtype=torch.float32)
        nat.mean_tokens(pf, VB, T, POSE_DIM, pooled)
        h1 = self._empty(VB, POSE_DIM, dtype=torch.float32)
        h2 = self._empty(VB, POSE_DIM, dtype=torch.float32)
        nat.linear_small(pooled, VB, POSE_DIM, w.pose_mlp[0][0], w.pose_mlp[0][1], POSE_DIM, nat.ACT_RELU, h1)
        nat.linear_small(h1, VB, POSE_DIM, w.pose_mlp[1][0], w.pose_mlp[1][1], POSE_DIM, nat.ACT_RELU, h2)
        raw = self._empty(VB, 7, dtype=torch.float32)
        nat.linear_small(h2, VB, POSE_DIM, w.pose_tr[0], w.pose_tr[1], 7, nat.ACT_NONE, raw)
        if taps is not None:
            taps["pose_raw"] = raw
        return raw

    def scale(self, tok, taps=None):
        """MLPHead (mlp_head.py:13-92) on the scale-token feature(s) (B, dim) -> raw (B,)."""
        w = self.w.scale_mlp
        m = tok.shape[0] if tok.dim() == 2 else 1
        a = self._empty(m, 196, dtype=torch.float32)
        b = self._empty(m, 196, dtype=torch.float32)
        nat.linear_small(tok, m, self.info.dim, w[0][0], w[0][1], 196, nat.ACT_NONE, a)
        nat.linear_small(a, m, 196, w[1][0], w[1][1], 196, nat.ACT_RELU, b)
        nat.linear_small(b, m, 196, w[2][0], w[2][1], 196, nat.ACT_RELU, a)
        raw = self._empty(m, dtype=torch.float32)
        nat.linear_small(a, m, 196, w[3][0], w[3][1], 1, nat.ACT_NONE, raw)
        if taps is not None:
            taps["scale_raw"] = raw
        return raw

    # ----------------------------------------------------------------------------------------------- run
    @torch.no_grad()
    def run(self, imgs: torch.Tensor, taps: Optional[dict] = None, shard=None, comm=None,
            geo: Optional[GeoInputs] = None, dpt_chunk: Optional[int] = None,
            pe_idx: Optional[torch.Tensor] = None, scenes: int = 1, fault=None) -> Dict[str, torch.Tensor]:
        """imgs: (V, 3, H, W) fp32 DINOv2-normalised on this device (B = 1 per view).  Returns the raw
        per-pixel / per-view outputs of MapAnything.forward, view-major.  With `shard`/`comm`, imgs are this
        rank's views only (parallel.ShardPlan.local_views) and the outputs are those views'.  `geo` carries the
        optional geometric inputs of these views (GeoInputs).  dpt_chunk: run the dense head over at most that many
        views at a time (memory_efficient_inference, model.py:1479-1516); None = all views at once.
        scenes = B > 1: imgs are B scenes of V views, scene-major ((B*V, 3, H, W), image b*V + v), run as one batch
        (the reference's batched forward, model.py:687-721): outputs scene-major, metric_scaling_factor (B, 1).
        fault: an armed _native.FaultSlot — the device fault word is published into it right after the transformer
        (the last LayerNorm-fused launch), so the caller can check it while the heads still run."""
        if imgs.dim() != 4 or imgs.shape[1] != 3:
            raise AssertionError("images must be (V, 3, H, W)")
        VB, _, H, W = imgs.shape
        if H % PATCH or W % PATCH:
            raise AssertionError(f"Input shape must be divisible by patch size: {PATCH}")
        imgs = imgs.to(self.device, torch.float32).contiguous()
        if fault is not None:  # the call's publish reports only the faults raised since here (stream order)
            with torch.cuda.device(self.device):
                fault.reset()
        B = scenes
        if B > 1 and ((geo is not None and geo.scenes != B) or taps is not None or VB % B
                      or (shard is not None and shard.scenes != B)):
            raise ValueError("batched scenes run without taps, with VB a multiple of B, a shard plan of B scenes and "
                             "geometric inputs batched the same way (GeoInputs.scenes)")
        with torch.cuda.device(self.device):
            fused_lp, fused_f32, (hp, wp) = self.encode(imgs, taps, geo, scenes=B)
            T = hp * wp
            if shard is not None and (shard.counts[shard.rank] * B != VB or shard.tokens_per_view != T):
                raise AssertionError("shard plan does not match the local views")
            if self.info.nonref_pe and pe_idx is None:
                raise ValueError("this info-sharing variant encodes every view's index: pass pe_idx")
            # DPT inputs (model.py:1724-1768): [encoder, tap0, tap1, final] or, with three taps, [tap0..2, final].
            # The fused encoder features enter the heads as a head operand (fp32 in the reference's heads); they are
            # split BEFORE the transformer when it has no input projection, because aat() then runs its residual
            # stream in place in fused_f32
            first = None
            if len(self.info.indices) != 3:
                if not self.hsplit:
                    first = fused_lp
                elif self.w.pe_proj is None:
                    first = self.head_rows(fused_f32[:VB * T])
            inter, fin_lp, tok = self.aat(fused_lp, VB, T, taps, shard=shard, comm=comm, pe_idx=pe_idx,
                                          fused_f32=fused_f32, scenes=B)
            # the device fault word is published after the transformer — or, when the TF32-equivalent heads can
            # raise MAPA_FAULT_F16_RANGE, once the last binary16 split operand exists: right before the regressor's
            # last conv (which writes fp32 outputs only), so ~1 ms of GPU work is still queued when the host sees
            # the slot and returns (run_heads; MAPA_FAULT_AT=transformer forces the early point, =end the very end)
            at = os.environ.get("MAPA_FAULT_AT", "last_conv")
            late = self.hfmt in ("f16", "f16x2") and self.hsplit and at != "transformer"
            if fault is not None and not late:
                fault.publish()
            if len(inter) == 3:
                first, l11, l17 = inter
            else:
                if first is None:
                    first = self.head_rows(fused_f32[:VB * T])
                l11, l17 = inter
            pending = [fault if late else None]
            out = self.run_heads(first, l11, l17, fin_lp, tok, VB, hp, wp, H, W, taps=taps, dpt_chunk=dpt_chunk,
                                 scenes=B, fault=pending if at != "end" else None)
            if pending[0] is not None:  # not published inside the heads (chunked dense head, unfused, "end")
                pending[0].publish()
            return out

    def run_heads(self, first, l11, l17, fin_lp, tok, VB, hp, wp, H, W, taps=None, dpt_chunk=None, scenes: int = 1,
                  fault=None):
        """downstream_head + output assembly (model.py:1774-1923): pose head on the final features, scale head on the
        scale-token feature, DPT + regressor + dense head on [first, l11, l17, final].  first / l11 / l17 / fin_lp are
        head operands (head_rows: split rows in the bf16 recipe, fp32 rows in fp32 mode; fin_lp may carry the scale
        tokens as its last rows); tok is the fp32 scale-token feature (B, dim) of the B = scenes scenes, whose VB = B x V
        images are scene-major."""
        T = hp * wp
        B = scenes
        V = VB // B
        with torch.cuda.device(self.device):
            pose_out = self._empty(VB, 19, dtype=torch.float32)
            scale = self._empty(B, dtype=torch.float32)
            poses44 = self._empty(VB, 4, 4, dtype=torch.float32)
            # one scale per image for the dense head when scenes are batched (image i: scale[i // V])
            scale_img = scale if B == 1 else self._empty(VB, dtype=torch.float32)
            # The pose and scale heads depend only on the transformer's outputs and feed only the last DPT conv (its
            # fused dense head): they run as a branch on a side stream, forked here and joined right before that conv,
            # so their small, under-filling launches (7 GEMMs over 301 tiles, pooling, MLPs) overlap the DPT's.
            # Every side-stream segment starts behind all earlier work of the main stream (wait_stream), and the
            # branch's own temporaries never leave it, so the caching allocator's per-stream reuse stays safe; the
            # outputs above are main-stream buffers.  Captured as a fork / join of the HIP graph.
            side = self._head_stream()
            cur = torch.cuda.current_stream(self.device)
            if side is not None:
                side.wait_stream(cur)
            with torch.cuda.stream(side if side is not None else cur):
                pose_raw = self.pose(fin_lp, VB, T, taps)
                scale_raw = self.scale(tok, taps)
                for b in range(B):  # each scene's views take its own metric scale
                    sl = slice(b * V, (b + 1) * V)
                    nat.pose_scale_finalize(pose_raw[sl], scale_raw[b:b + 1], V, 1, pose_out[sl], scale[b:b + 1],
                                            poses44[sl])
                if B > 1:
                    scale_img.view(B, V).copy_(scale.view(B, 1).expand(B, V))
            joined = [side is None]

            one_pass = not dpt_chunk or int(dpt_chunk) >= VB

            def join():  # before the last conv of the (single-pass) dense head: its inputs are all written by then
                if one_pass and fault is not None and fault[0] is not None:
                    if not joined[0]:
                        cur.wait_stream(side)
                        joined[0] = True
                    fault[0].publish()  # the last binary16 split operand exists (run())
                    fault[0] = None
                if not joined[0]:
                    cur.wait_stream(side)
                    joined[0] = True
            f = torch.float32
            out = dict(
                pts3d=self._empty(VB, H, W, 3, dtype=f), pts3d_cam=self._empty(VB, H, W, 3, dtype=f),
                ray_directions=self._empty(VB, H, W, 3, dtype=f), depth_along_ray=self._empty(VB, H, W, 1, dtype=f),
                conf=self._empty(VB, H, W, dtype=f), non_ambiguous_mask_logits=self._empty(VB, H, W, dtype=f),
                non_ambiguous_mask=self._empty(VB, H, W, dtype=torch.bool))  # kernel writes 0/1 bytes
            chunk = VB if not dpt_chunk else max(1, min(int(dpt_chunk), VB))
            fuse = self.fused_head_out()
            for v0 in range(0, VB, chunk):
                n = min(chunk, VB - v0)
                r0, r1 = v0 * T, (v0 + n) * T
                # (pose rows, scales, images per scale value) of these images
                sc = (scale, n) if B == 1 else (scale_img[v0:v0 + n], 1)
                outs = tuple(out[k][v0:v0 + n] for k in ("pts3d", "pts3d_cam", "ray_directions", "depth_along_ray",
                                                         "conf", "non_ambiguous_mask_logits", "non_ambiguous_mask"))
                hid = self.dpt(first[r0:r1], l11[r0:r1], l17[r0:r1], fin_lp[r0:r1], n, hp, wp, H, W,
                               taps if n == VB else None, head=(pose_out[v0:v0 + n],) + sc + outs if fuse else None,
                               join=join)
                if not fuse:  # the unfused head's batch = scales: scale[i % batch] (one scale, or one per image)
                    join()
                    nat.dense_head_out(hid, n, H * W, self.w.reg_w6, self.w.reg_b6, pose_out[v0:v0 + n], sc[0],
                                       1 if B == 1 else n, *outs)
                del hid
            join()
            out["cam_trans"] = pose_out[:, 0:3]
            out["cam_quats"] = pose_out[:, 3:7]
            out["metric_scaling_factor"] = scale.view(B, 1)
            out["camera_poses"] = poses44
        return out

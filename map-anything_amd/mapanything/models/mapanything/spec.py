"""State-dict layout of the released MapAnything architecture (configs/inference.json).

Restates the parameter names/shapes that `MapAnything.__init__` (model.py:99-231) creates for the released
config: DINOv2 ViT-L/14 (vision_transformer.py:57-199, 420-431; mask_token deleted at dinov2.py:93-95), the
geometric-input encoders (dense_rep_encoder.py:55-287, global_rep_encoder.py:14-100), fusion LayerNorm, scale
token, AAT-IFR (alternating_attention_transformer.py:22-175), DPT feature + regression heads (dpt.py:32-311,
dpt_block.py:21-255), pose head (pose_head.py:50-159) and scale head (mlp_head.py:13-92).

`canonical_spec()` lists each tensor once; `ALIASES` maps the extra state-dict keys that share storage with a
canonical tensor (`dense_head.0/1.*`, `scratch.layer_rn.N`, `input_process.N.1`), so a checkpoint written by the
reference can be read either way.
"""

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

Spec = List[Tuple[str, Tuple[int, ...]]]

ENC_DIM = 1024
ENC_DEPTH = 24
ENC_MLP = 4096
PATCH = 14
AAT_DIM = 768
AAT_DEPTH = 24
AAT_MLP = 3072
DPT_LAYER_DIMS = (96, 192, 384, 768)
DPT_FEAT = 256
POSE_DIM = 4 * PATCH * PATCH  # 784


@dataclass(frozen=True)
class InfoSharingSpec:
    """The multi-view transformer variant of an info_sharing_config (model.py:240-330 picks the class):

    * kind "alternating" = MultiViewAlternatingAttentionTransformerIFR (alternating_attention_transformer.py:386-771:
      even blocks attend over every view + the additional tokens, odd blocks inside each view without them);
      "global" = MultiViewGlobalAttentionTransformerIFR (global_attention_transformer.py:347-640: every block global).
    * view positional encoding from the sinusoid `view_pos_table` (pe_rows rows): row 0 on the reference view when
      ref_pe; rows 1.. (sequential, or torch.randint(1, pe_rows) per forward when rand_idx) on the other views when
      nonref_pe.  AAT: ref_pe = distinguish_ref_and_non_ref_views, nonref_pe = that and use_pe_for_non_reference_views,
      table rows max_num_views_for_pe if nonref_pe else 1 (alternating_attention_transformer.py:159-172, 594-620);
      GAT: both always, max_num_views rows (global_attention_transformer.py:160-167, 543-563).
    * attention logit scaling (transformer_blocks.py:185-196), applied to q per block with N = that block's tokens:
      scalable softmax x ln N; entropy scaling x sqrt(growth * ln N / ln base).
    """
    kind: str = "alternating"
    depth: int = 24
    dim: int = AAT_DIM      # 1024 / 16 heads in the 48-layer configs (proj_embed is then the identity)
    heads: int = 12
    indices: Tuple[int, ...] = (11, 17)  # 2 taps (DPT also reads the encoder features) or 3 (it does not)
    ref_pe: bool = True
    nonref_pe: bool = False
    rand_idx: bool = True
    pe_rows: int = 1
    scalable_softmax: bool = False
    entropy_scaling: bool = False
    entropy_base: int = 444
    entropy_growth: float = 1.4

    @staticmethod
    def from_config(info_sharing_config: Optional[Dict]) -> "InfoSharingSpec":
        if not info_sharing_config:
            return InfoSharingSpec()
        a = info_sharing_config.get("module_args", {})
        kind = "global" if info_sharing_config.get("model_type") == "global_attention" else "alternating"
        common = dict(depth=int(a.get("depth", 12)), dim=int(a.get("dim", 768)), heads=int(a.get("num_heads", 12)),
                      indices=tuple(int(i) for i in a.get("indices", (11, 17))),
                      scalable_softmax=bool(a.get("use_scalable_softmax", False)),
                      entropy_scaling=bool(a.get("use_entropy_scaling", False)),
                      entropy_base=int(a.get("base_token_count_for_entropy_scaling", 444)),
                      entropy_growth=float(a.get("entropy_scaling_growth_factor", 1.4)))
        if kind == "global":
            return InfoSharingSpec(kind=kind, ref_pe=True, nonref_pe=True,
                                   rand_idx=bool(a["use_rand_idx_pe_for_non_reference_views"]),
                                   pe_rows=int(a["max_num_views"]), **common)
        ref = bool(a.get("distinguish_ref_and_non_ref_views", True))
        nonref = ref and bool(a.get("use_pe_for_non_reference_views", False))
        return InfoSharingSpec(kind=kind, ref_pe=ref, nonref_pe=nonref,
                               rand_idx=bool(a.get("use_rand_idx_pe_for_non_reference_views", True)),
                               pe_rows=int(a.get("max_num_views_for_pe", 1000)) if nonref else 1, **common)

    def is_global(self, d: int) -> bool:
        return self.kind == "global" or d % 2 == 0

    def q_scale(self, n_tokens: int) -> float:
        """Multiplier on q (on top of SDPA's head_dim^-0.5) for a block over n_tokens tokens."""
        f = 1.0
        if self.scalable_softmax:
            f *= math.log(n_tokens)
        if self.entropy_scaling:
            f *= math.sqrt(self.entropy_growth * math.log(n_tokens) / math.log(self.entropy_base))
        return f


RELEASED_INFO = InfoSharingSpec()


def _linear(spec: Spec, name: str, out_f: int, in_f: int, bias: bool = True):
    spec.append((f"{name}.weight", (out_f, in_f)))
    if bias:
        spec.append((f"{name}.bias", (out_f,)))


def _conv(spec: Spec, name: str, out_c: int, in_c: int, k: int, bias: bool = True):
    spec.append((f"{name}.weight", (out_c, in_c, k, k)))
    if bias:
        spec.append((f"{name}.bias", (out_c,)))


def _ln(spec: Spec, name: str, dim: int):
    spec.append((f"{name}.weight", (dim,)))
    spec.append((f"{name}.bias", (dim,)))


def _dense_rep_encoder(spec: Spec, name: str, in_chans: int):
    dims = (588, 768, 1024)
    _conv(spec, f"{name}.conv_in", dims[0], in_chans * PATCH * PATCH, 3)
    for i in range(2):
        _conv(spec, f"{name}.encoder.{i}.conv1", dims[i + 1], dims[i], 3)
        _conv(spec, f"{name}.encoder.{i}.conv2", dims[i + 1], dims[i + 1], 3)
        _conv(spec, f"{name}.encoder.{i}.shortcut", dims[i + 1], dims[i], 1)
    _conv(spec, f"{name}.encoder.2", ENC_DIM, dims[-1], 1)
    _ln(spec, f"{name}.norm_layer", ENC_DIM)


def _global_rep_encoder(spec: Spec, name: str, in_chans: int):
    _linear(spec, f"{name}.encoder.0.0.0.0", 128, in_chans)
    _linear(spec, f"{name}.encoder.0.0.1", 256, 128)
    _linear(spec, f"{name}.encoder.0.1", 512, 256)
    _linear(spec, f"{name}.encoder.1", ENC_DIM, 512)
    _ln(spec, f"{name}.norm_layer", ENC_DIM)


def _rcu(spec: Spec, name: str):
    _conv(spec, f"{name}.conv1", DPT_FEAT, DPT_FEAT, 3)
    _conv(spec, f"{name}.conv2", DPT_FEAT, DPT_FEAT, 3)


def canonical_spec(info: InfoSharingSpec = RELEASED_INFO) -> Spec:
    s: Spec = []
    s.append(("scale_token", (ENC_DIM,)))
    # DINOv2 ViT-L/14
    s.append(("encoder.model.cls_token", (1, 1, ENC_DIM)))
    s.append(("encoder.model.pos_embed", (1, 37 * 37 + 1, ENC_DIM)))
    _conv(s, "encoder.model.patch_embed.proj", ENC_DIM, 3, PATCH)
    for b in range(ENC_DEPTH):
        p = f"encoder.model.blocks.{b}"
        _ln(s, f"{p}.norm1", ENC_DIM)
        _linear(s, f"{p}.attn.qkv", 3 * ENC_DIM, ENC_DIM)
        _linear(s, f"{p}.attn.proj", ENC_DIM, ENC_DIM)
        s.append((f"{p}.ls1.gamma", (ENC_DIM,)))
        _ln(s, f"{p}.norm2", ENC_DIM)
        _linear(s, f"{p}.mlp.fc1", ENC_MLP, ENC_DIM)
        _linear(s, f"{p}.mlp.fc2", ENC_DIM, ENC_MLP)
        s.append((f"{p}.ls2.gamma", (ENC_DIM,)))
    _ln(s, "encoder.model.norm", ENC_DIM)
    # geometric-input encoders
    _dense_rep_encoder(s, "ray_dirs_encoder", 3)
    _dense_rep_encoder(s, "depth_encoder", 1)
    _global_rep_encoder(s, "depth_scale_encoder", 1)
    _global_rep_encoder(s, "cam_rot_encoder", 4)
    _global_rep_encoder(s, "cam_trans_encoder", 3)
    _global_rep_encoder(s, "cam_trans_scale_encoder", 1)
    _ln(s, "fusion_norm_layer", ENC_DIM)
    # AAT
    D = info.dim
    if info.ref_pe:
        s.append(("info_sharing.view_pos_table", (info.pe_rows, D)))
    if D != ENC_DIM:  # nn.Identity otherwise (alternating_attention_transformer.py:121-124)
        _linear(s, "info_sharing.proj_embed", D, ENC_DIM)
    for b in range(info.depth):
        p = f"info_sharing.self_attention_blocks.{b}"
        _ln(s, f"{p}.norm1", D)
        _linear(s, f"{p}.attn.qkv", 3 * D, D)
        _linear(s, f"{p}.attn.proj", D, D)
        _ln(s, f"{p}.norm2", D)
        _linear(s, f"{p}.mlp.fc1", 4 * D, D)
        _linear(s, f"{p}.mlp.fc2", D, 4 * D)
    _ln(s, "info_sharing.norm", D)
    # DPT feature head
    h = "dpt_feature_head"
    # three info-sharing taps feed the DPT without the encoder features (model.py:362-372)
    in_dims = (D if len(info.indices) == 3 else ENC_DIM, D, D, D)
    for i, ld in enumerate(DPT_LAYER_DIMS):
        s.append((f"{h}.scratch.layer{i + 1}_rn.weight", (DPT_FEAT, ld, 3, 3)))
    for r in (1, 2, 3, 4):
        _conv(s, f"{h}.scratch.refinenet{r}.out_conv", DPT_FEAT, DPT_FEAT, 1)
        if r != 4:
            _rcu(s, f"{h}.scratch.refinenet{r}.resConfUnit1")
        _rcu(s, f"{h}.scratch.refinenet{r}.resConfUnit2")
    _conv(s, f"{h}.input_process.0.0.0", DPT_LAYER_DIMS[0], in_dims[0], 1)
    s.append((f"{h}.input_process.0.0.1.weight", (DPT_LAYER_DIMS[0], DPT_LAYER_DIMS[0], 4, 4)))
    s.append((f"{h}.input_process.0.0.1.bias", (DPT_LAYER_DIMS[0],)))
    _conv(s, f"{h}.input_process.1.0.0", DPT_LAYER_DIMS[1], in_dims[1], 1)
    s.append((f"{h}.input_process.1.0.1.weight", (DPT_LAYER_DIMS[1], DPT_LAYER_DIMS[1], 2, 2)))
    s.append((f"{h}.input_process.1.0.1.bias", (DPT_LAYER_DIMS[1],)))
    _conv(s, f"{h}.input_process.2.0.0", DPT_LAYER_DIMS[2], in_dims[2], 1)
    _conv(s, f"{h}.input_process.3.0.0", DPT_LAYER_DIMS[3], in_dims[3], 1)
    _conv(s, f"{h}.input_process.3.0.1", DPT_LAYER_DIMS[3], DPT_LAYER_DIMS[3], 3)
    # DPT regressor
    _conv(s, "dpt_regressor_head.conv1", 128, DPT_FEAT, 3)
    _conv(s, "dpt_regressor_head.conv2.0", 128, 128, 3)
    _conv(s, "dpt_regressor_head.conv2.2", 6, 128, 1)
    # pose head
    _conv(s, "pose_head.proj", POSE_DIM, D, 1)
    for b in range(2):
        for c in (1, 2, 3):
            _conv(s, f"pose_head.res_conv.{b}.res_conv{c}", POSE_DIM, POSE_DIM, 1)
    _linear(s, "pose_head.more_mlps.0", POSE_DIM, POSE_DIM)
    _linear(s, "pose_head.more_mlps.2", POSE_DIM, POSE_DIM)
    _linear(s, "pose_head.fc_t", 3, POSE_DIM)
    _linear(s, "pose_head.fc_rot", 4, POSE_DIM)
    # scale head
    _linear(s, "scale_head.proj", 196, D)
    _linear(s, "scale_head.mlp.0.0", 196, 196)
    _linear(s, "scale_head.mlp.1.0", 196, 196)
    _linear(s, "scale_head.output_proj", 1, 196)
    return s


def aliases(info: InfoSharingSpec = RELEASED_INFO) -> Dict[str, str]:
    """alias key -> canonical key (tensors that share storage in the reference's state dict)."""
    out: Dict[str, str] = {}
    h = "dpt_feature_head"
    feat_alias = {}
    for i in range(4):
        feat_alias[f"scratch.layer_rn.{i}.weight"] = f"scratch.layer{i + 1}_rn.weight"
        feat_alias[f"input_process.{i}.1.weight"] = f"scratch.layer{i + 1}_rn.weight"
    for a, c in feat_alias.items():
        out[f"{h}.{a}"] = f"{h}.{c}"
        out[f"dense_head.0.{a}"] = f"{h}.{c}"
    for n, _ in canonical_spec(info):
        if n.startswith(h + "."):
            out["dense_head.0." + n[len(h) + 1:]] = n
        elif n.startswith("dpt_regressor_head."):
            out["dense_head.1." + n[len("dpt_regressor_head."):]] = n
    return out


def full_spec(info: InfoSharingSpec = RELEASED_INFO) -> Spec:
    """Every key of the reference's state_dict (canonical + aliases)."""
    canon = canonical_spec(info)
    shapes = dict(canon)
    return canon + [(a, shapes[c]) for a, c in aliases(info).items()]

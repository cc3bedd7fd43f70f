"""`MapAnything` — drop-in for `mapanything.models.MapAnything` (reference model.py:96-2355) on MI355X.

Same constructor config (configs/inference.json schema), same `from_pretrained(local_dir)`, `infer(views, ...)`
keyword arguments and output dictionaries (model.py:2206-2355), same `forward(views)` raw outputs
(model.py:1657-2152), same `ValueError`s for invalid views (inference.py:146-217).  Every arithmetic step runs in
the gfx950 HIP library (`MapaEngine`); this class is host glue: validation, device placement, bookkeeping.

Differences that are by design:
  * weights come from a LOCAL directory (config.json + model.safetensors) or the synthetic named-PRNG
    checkpoint; there is no hub download (no network on this box),
  * `precision="bf16"` (default) mirrors `infer(use_amp=True, amp_dtype="bf16")` (`amp_dtype="fp16"` the same on
    fp16 operands) — bf16 encoder/transformer, the
    geometric encoders and the downstream heads as the reference runs them with autocast disabled (model.py:1377,
    1774): the geometric encoders fp32-exact (split-precision bf16 GEMMs on MI355X), the heads by default
    (`head_precision="tf32"`) at the precision the reference's fp32 head convs / linears get on its own GPUs — TF32
    (cudnn's default; matmul.allow_tf32 = True at model.py:93): both operands rounded to 11 significant bits, fp32
    accumulation — as binary16 operands (the same 11 bits; `"tf32x2"` keeps 22 bits of each activation as a binary16
    [hi | lo] pair at twice the work); `head_precision="fp32"` keeps the
    fp32-exact split-bf16 heads (the default of the fp16 recipe, amp_dtype="fp16", whose transformer rounds 8x finer
    than bf16: its tolerance is the reference's own fp16 spread measured with exact fp32 heads); `use_amp=False` (or precision="fp32") runs the exact-fp32 MFMA path;
    `head_precision="bf16"` is an opt-in fast mode with bf16 heads (not the reference's recipe),
  * B > 1 scenes per view (the reference's batch_size_per_view, model.py:687): the scenes run as ONE engine call
    (encoder, geometric encoders, frame layers and heads over all B x V images, global attention, scale token and
    scale head per scene, as the reference's batched forward, model.py:687-721); on a view-sharded model every rank
    runs its views of all B scenes.  The per-view outputs are concatenated on the batch dimension as the reference
    returns them.
"""

from __future__ import annotations

import json
import os
import warnings
from collections import OrderedDict
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ... import _native as nat
from ...parallel import comm_timeout, force_collectives, force_overlap
from ...utils.inference import (postprocess_outputs, preprocess_input_views_for_inference,
                                validate_input_views_for_inference)
from .spec import InfoSharingSpec, aliases, canonical_spec, full_spec

SUPPORTED = dict(
    encoder="dinov2", size="large", info_sharing=("alternating_attention", "global_attention"),
    return_type="intermediate_features", pred_head="dpt+pose", adaptor="raydirs+depth+pose+confidence+mask",
)


def _check_config(encoder_config, info_sharing_config, pred_head_config):
    problems = []
    if encoder_config.get("encoder_str") != "dinov2" or encoder_config.get("size", "large") != "large":
        problems.append(f"encoder {encoder_config.get('encoder_str')}/{encoder_config.get('size')}")
    if encoder_config.get("with_registers", False):
        problems.append("dinov2 with registers")
    if info_sharing_config.get("model_type") not in SUPPORTED["info_sharing"]:
        problems.append(f"info_sharing {info_sharing_config.get('model_type')}")
    if info_sharing_config.get("model_return_type") != SUPPORTED["return_type"]:
        problems.append(f"return type {info_sharing_config.get('model_return_type')}")
    args = info_sharing_config.get("module_args", {})
    depth = int(args.get("depth", 12))
    idx = list(args.get("indices", []))
    if (len(idx) not in (2, 3) or not all(0 <= int(i) < depth for i in idx)
            or any(int(a) >= int(b) for a, b in zip(idx, idx[1:]))):
        problems.append(f"info-sharing intermediate indices {idx} (2 or 3 increasing block indices < depth)")
    dim, heads = int(args.get("dim", 768)), int(args.get("num_heads", 12))
    if heads <= 0 or dim != 64 * heads or float(args.get("mlp_ratio", 4.0)) != 4.0:
        # the attention kernels are built for 64-wide heads (768/12 and the 48-layer 1024/16)
        problems.append(f"info-sharing dim {dim} / {heads} heads / mlp_ratio {args.get('mlp_ratio', 4.0)}")
    if (info_sharing_config.get("custom_positional_encoding") is not None
            or args.get("custom_positional_encoding") is not None):
        # RoPE-2D: with MapAnything's scale token the reference adds a list of None positions to the position
        # tensor (alternating_attention_transformer.py:294, global_attention_transformer.py:541) and fails
        problems.append("custom positional encoding (RoPE)")
    if args.get("qk_norm", False):
        problems.append("qk_norm")
    if pred_head_config.get("type") != SUPPORTED["pred_head"]:
        problems.append(f"pred head {pred_head_config.get('type')}")
    if pred_head_config.get("adaptor_type") != SUPPORTED["adaptor"]:
        problems.append(f"adaptor {pred_head_config.get('adaptor_type')}")
    if problems:
        raise ValueError("MapAnything (MI355X engine) implements the released architecture "
                         f"(configs/inference.json); unsupported: {', '.join(problems)}")


class MapAnything:
    """Modular MapAnything model (reference model.py:96) — MI355X-native inference engine."""

    def __init__(self, name: str, encoder_config: Dict, info_sharing_config: Dict, pred_head_config: Dict,
                 geometric_input_config: Dict, fusion_norm_layer=None, pretrained_checkpoint_path: str = None,
                 load_specific_pretrained_submodules: bool = False, specific_pretrained_submodules: list = None,
                 torch_hub_force_reload: bool = False, precision: str = "bf16", hip_graphs: bool = True,
                 head_precision: Optional[str] = None):
        _check_config(encoder_config, info_sharing_config, pred_head_config)
        self.info = InfoSharingSpec.from_config(info_sharing_config)
        self.name = name
        self.encoder_config = encoder_config
        self.info_sharing_config = info_sharing_config
        self.pred_head_config = pred_head_config
        self.geometric_input_config = dict(geometric_input_config)
        self.class_init_args = dict(name=name, encoder_config=encoder_config, info_sharing_config=info_sharing_config,
                                    pred_head_config=pred_head_config, geometric_input_config=geometric_input_config,
                                    pretrained_checkpoint_path=pretrained_checkpoint_path,
                                    load_specific_pretrained_submodules=load_specific_pretrained_submodules,
                                    specific_pretrained_submodules=specific_pretrained_submodules,
                                    torch_hub_force_reload=torch_hub_force_reload)
        self.precision = precision
        if head_precision not in (None, "tf32", "tf32x2", "fp32", "bf16"):
            raise ValueError(f"head_precision must be 'tf32', 'tf32x2', 'fp32' or 'bf16' (None: the recipe's default), "
                             f"got {head_precision}")
        self.head_precision = head_precision  # None: "tf32" under bf16 autocast, "fp32" under fp16 autocast
        self._sd: Optional[Dict[str, np.ndarray]] = None
        self._engines: Dict[tuple, Any] = {}
        self._device = torch.device("cpu")
        self._comm = None
        self._gather = None
        self.training = False
        # Replay the engine's ~350 launches per forward from a captured HIP graph (image-only, single device,
        # all views in one dense-head pass): removes the host launch gaps.  MAPA_HIP_GRAPHS=0 disables.
        self.hip_graphs = hip_graphs and os.environ.get("MAPA_HIP_GRAPHS", "1") != "0"
        self._graphs: "OrderedDict[tuple, tuple]" = OrderedDict()
        # sharded capture (the collectives through the direct RCCL communicator, parallel.RcclComm, inside the HIP
        # graph): off with MAPA_SHARD_GRAPHS=0 (eager launches, collectives through the process group and its
        # watchdog), or on every rank once any rank's capture has failed
        self._shard_graphs = os.environ.get("MAPA_SHARD_GRAPHS", "1") != "0"
        # why the sharded path runs eagerly (None while sharded graphs are on); bench.py reports it
        self.shard_graph_fallback: Optional[str] = None if self._shard_graphs else "MAPA_SHARD_GRAPHS=0"
        self._modules: Dict[str, Any] = {}
        if pretrained_checkpoint_path is not None:
            self.load_checkpoint(pretrained_checkpoint_path)

    # ------------------------------------------------------------------------------------------ weights
    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, local_files_only: bool = True, **kwargs):
        """Local-directory version of PyTorchModelHubMixin.from_pretrained (config.json + model.safetensors)."""
        path = pretrained_model_name_or_path
        if not os.path.isdir(path):
            raise FileNotFoundError(
                f"{path!r} is not a local directory: this engine loads config.json + model.safetensors from disk "
                "(no hub access); download the checkpoint elsewhere and pass its directory")
        with open(os.path.join(path, "config.json")) as f:
            cfg = json.loads(_strip_comments(f.read()))
        cfg.update({k: v for k, v in kwargs.items() if k in ("precision", "head_precision", "hip_graphs")})
        model = cls(**cfg)
        st = os.path.join(path, "model.safetensors")
        if os.path.exists(st):
            from safetensors.numpy import load_file
            model.load_state_dict(load_file(st))
        else:
            raise FileNotFoundError(f"{st} not found")
        return model

    @classmethod
    def from_config_file(cls, path: str, **kwargs):
        with open(path) as f:
            cfg = json.loads(_strip_comments(f.read()))
        cfg.update(kwargs)
        return cls(**cfg)

    def load_checkpoint(self, path: str):
        """`_load_pretrained_weights` (model.py:636-666): a torch checkpoint with a 'model' state dict."""
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        self.load_state_dict(ckpt["model"] if "model" in ckpt else ckpt)

    def load_state_dict(self, state_dict: Dict[str, Any], strict: bool = True):
        canon = dict(canonical_spec(self.info))
        al = aliases(self.info)
        sd: Dict[str, np.ndarray] = {}
        for k, v in state_dict.items():
            arr = v.detach().float().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v, np.float32)
            key = al.get(k, k)
            if key not in canon:
                if strict:
                    raise KeyError(f"unexpected key in state_dict: {k}")
                continue
            if tuple(arr.shape) != tuple(canon[key]):
                raise ValueError(f"shape mismatch for {k}: {arr.shape} vs {canon[key]}")
            sd[key] = arr
        missing = [k for k in canon if k not in sd]
        if missing and strict:
            raise KeyError(f"missing keys in state_dict: {missing[:5]} ... ({len(missing)})")
        self._sd = sd
        self._engines.clear()
        self._graphs.clear()
        self._modules.clear()
        return self

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        """nn.Module.state_dict() of the reference model (model.py:96): every key the reference's state dict has —
        the canonical tensors and the alias keys of the shared DPT modules (`dense_head.0/1.*`,
        `scratch.layer_rn.N`, `input_process.N.1`), which share storage as in the reference — as fp32 CPU tensors."""
        if self._sd is None:
            raise RuntimeError("no weights loaded")
        canon = {k: torch.from_numpy(v) for k, v in self._sd.items()}
        al = aliases(self.info)
        return OrderedDict((name, canon[al.get(name, name)]) for name, _ in full_spec(self.info))

    def named_parameters(self):
        """(name, tensor) once per distinct tensor (nn.Module de-duplicates shared parameters the same way)."""
        if self._sd is None:
            raise RuntimeError("no weights loaded")
        for name, _ in canonical_spec(self.info):
            yield name, torch.from_numpy(self._sd[name])

    def parameters(self):
        for _, t in self.named_parameters():
            yield t

    def save_pretrained(self, save_directory: str):
        """PyTorchModelHubMixin.save_pretrained layout: config.json (the constructor config) + model.safetensors
        (one entry per distinct tensor, as safetensors' save_model de-duplicates shared storage)."""
        from safetensors.numpy import save_file

        if self._sd is None:
            raise RuntimeError("no weights loaded")
        os.makedirs(save_directory, exist_ok=True)
        cfg = {k: v for k, v in self.class_init_args.items() if v is not None}
        with open(os.path.join(save_directory, "config.json"), "w") as f:
            json.dump(cfg, f, indent=1)
        save_file({k: np.ascontiguousarray(v) for k, v in self._sd.items()},
                  os.path.join(save_directory, "model.safetensors"))

    def load_synthetic_weights(self):
        """Named-PRNG synthetic checkpoint (mapanything/utils/synthetic.py) — bench/tests only."""
        from ...utils.synthetic import synthetic_state_dict

        self._sd = synthetic_state_dict(canonical_spec(self.info))
        self._engines.clear()
        self._graphs.clear()
        self._modules.clear()
        return self

    # ------------------------------------------------------- sub-modules (uniception dataclass contracts, modules.py)
    def _module(self, name: str):
        m = self._modules.get(name)
        if m is None:
            from . import modules as M

            make = {"encoder": M.DINOv2Encoder, "info_sharing": M.MultiViewAlternatingAttentionTransformerIFR,
                    "dpt_feature_head": M.DPTFeature, "dpt_regressor_head": M.DPTRegressionProcessor,
                    "dense_adaptor": M.RayDirectionsPlusDepthWithConfidenceAndMaskAdaptor,
                    "pose_head": M.PoseHead, "pose_adaptor": M.CamTranslationPlusQuatsAdaptor,
                    "scale_head": M.MLPHead, "scale_adaptor": M.ScaleAdaptor, "fusion_norm_layer": M.FusionNorm}
            if name == "dense_head":
                m = M.DenseHead(self.dpt_feature_head, self.dpt_regressor_head)
            else:
                m = make[name](self)
            self._modules[name] = m
        return m

    encoder = property(lambda self: self._module("encoder"))                        # model.py:168-172
    info_sharing = property(lambda self: self._module("info_sharing"))              # model.py:316
    dpt_feature_head = property(lambda self: self._module("dpt_feature_head"))      # model.py:394
    dpt_regressor_head = property(lambda self: self._module("dpt_regressor_head"))  # model.py:395
    dense_head = property(lambda self: self._module("dense_head"))                  # model.py:398
    dense_adaptor = property(lambda self: self._module("dense_adaptor"))            # model.py:470
    pose_head = property(lambda self: self._module("pose_head"))                    # model.py:403
    pose_adaptor = property(lambda self: self._module("pose_adaptor"))
    scale_head = property(lambda self: self._module("scale_head"))                  # model.py:420
    scale_adaptor = property(lambda self: self._module("scale_adaptor"))            # model.py:634
    fusion_norm_layer = property(lambda self: self._module("fusion_norm_layer"))    # model.py:213

    @property
    def scale_token(self) -> torch.Tensor:
        """The learned scale token (1024,) fp32 on the model's device (model.py:218)."""
        return self.engine().w.scale_token.reshape(-1)

    # ------------------------------------------------------------------------------------ nn.Module-ish
    def to(self, device=None, *args, **kwargs):
        if device is not None:
            self._device = torch.device(device)
            if self._device.type == "cuda" and self._device.index is None:
                self._device = torch.device("cuda", torch.cuda.current_device())
        return self

    def cuda(self, device=None):
        return self.to(torch.device("cuda", device) if device is not None else "cuda")

    def eval(self):
        self.training = False
        return self

    def train(self, mode: bool = True):
        if mode:
            raise NotImplementedError("training is out of scope for the MI355X inference engine")
        return self.eval()

    @property
    def device(self) -> torch.device:
        return self._device

    def heads_for(self, precision: str) -> str:
        """The head precision a run at `precision` uses: head_precision, or by default 'tf32' (the reference's GPU
        recipe) under bf16 autocast and 'fp32' under the fp16 recipe; exact fp32 throughout at precision 'fp32'."""
        if precision == "fp32":
            return "fp32"
        if self.head_precision is not None:
            return self.head_precision
        return "fp32" if precision == "fp16" else "tf32"

    def engine(self, precision: Optional[str] = None, heads: Optional[str] = None):
        """The engine of a run at `precision` (heads: override heads_for(precision), e.g. the fp32-exact heads of the
        binary16 range fallback)."""
        prec = precision or self.precision
        if self._sd is None:
            raise RuntimeError("no weights loaded: use from_pretrained(local_dir), load_state_dict() or "
                               "load_synthetic_weights()")
        if self._device.type != "cuda":
            raise nat.NativeError("MapAnything (MI355X engine) runs on a gfx950 device only: call .to('cuda')")
        heads = heads if heads is not None and prec != "fp32" else self.heads_for(prec)
        key = (str(self._device), prec, heads)
        if key not in self._engines:
            from .engine import MapaEngine
            self._engines[key] = MapaEngine(self._sd, self._device, prec, self.info, heads=heads)
        return self._engines[key]

    def enable_view_sharding(self, group=None, comm=None, gather_outputs: Optional[str] = None):
        """Shard the views over the ranks of `group` (one process per GPU, torch.distributed over RCCL) or of an
        explicit communicator (parallel.ThreadComm in tests).  infer()/forward() then run only this rank's views.
        gather_outputs: None -> the returned list holds this rank's views' outputs and None for the others;
        "rank0" -> rank 0 returns every view's outputs, as the reference's infer does (model.py:2266-2282), the
        other ranks their own views'; "all" -> every rank returns every view's outputs."""
        import torch.distributed as dist

        from ...parallel import DistComm, RcclComm

        if gather_outputs not in (None, "rank0", "all"):
            raise ValueError(f"gather_outputs must be None, 'rank0' or 'all', got {gather_outputs!r}")
        if getattr(self, "_comm_dead", None):
            # a fresh communicator after an abort (_comm_failed): sharded HIP graphs are allowed again
            self._shard_graphs = os.environ.get("MAPA_SHARD_GRAPHS", "1") != "0"
            self.shard_graph_fallback = None if self._shard_graphs else "MAPA_SHARD_GRAPHS=0"
        if comm is None:
            comm = DistComm(group)
            if self._shard_graphs and dist.get_backend(group) == "nccl":
                # an RCCL group with sharded HIP graphs on: the collectives go to RCCL directly (capturable); every
                # rank keeps the process-group communicator instead if any rank's RCCL communicator fails
                dev = self._device if self._device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
                rc, err = None, None
                try:
                    rc = RcclComm(group, dev)
                except Exception as e:  # noqa: BLE001 -- agreed on below
                    err = e
                if comm.all_agree(rc is not None, dev):
                    comm = rc
                else:
                    warnings.warn(f"direct RCCL communicator unavailable ({err or 'on another rank'}); the sharded "
                                  "path runs eagerly on the process group")
                    self._shard_graphs = False
                    self.shard_graph_fallback = f"direct RCCL communicator unavailable: {err or 'on another rank'}"
        old = getattr(self, "_comm", None)
        if old is not None and old is not comm:
            # graphs captured against the previous communicator hold its RCCL handle: drop them, then release it
            for k in [k for k in self._graphs if k[-1] is not None]:
                del self._graphs[k]
            if hasattr(old, "close"):
                old.close()
        self._comm = comm
        self._gather = gather_outputs
        self._comm_dead = None
        return self

    # ------------------------------------------------------------------------------------------ forward
    def _check_views(self, views):
        for i, v in enumerate(views):
            if "img" not in v:
                # the reference's _encode_n_views (model.py:700) indexes views[i]["img"] for every view
                raise KeyError(f"view {i}: 'img'")
        B = views[0]["img"].shape[0]
        if any(v["img"].shape[0] != B for v in views):
            raise ValueError("every view must carry the same batch size (batch_size_per_view, model.py:687)")
        return B

    @staticmethod
    def _scene_views(views, b: int, B: int):
        """Scene b of a batch of B scenes: every per-sample entry of every view sliced to [b:b+1] (tensors and
        tuples of tensors with a leading B, lists of B entries); other entries are shared."""
        out = []
        for v in views:
            d = {}
            for k, x in v.items():
                if isinstance(x, torch.Tensor) and x.dim() >= 1 and x.shape[0] == B:
                    d[k] = x[b:b + 1]
                elif (isinstance(x, tuple) and x and all(isinstance(t, torch.Tensor) and t.dim() >= 1
                                                         and t.shape[0] == B for t in x)):
                    d[k] = tuple(t[b:b + 1] for t in x)
                elif isinstance(x, list) and len(x) == B:
                    d[k] = x[b:b + 1]
                else:
                    d[k] = x
            out.append(d)
        return out

    @staticmethod
    def _merge_scenes(per_scene):
        """[scene][view] output dicts -> [view] dicts with every entry concatenated over the scenes (dim 0), the
        reference's (B, ...) per-view outputs (model.py:1865-1923, 2266-2282)."""
        merged = []
        for i in range(len(per_scene[0])):
            if per_scene[0][i] is None:  # a view owned by another rank (view sharding)
                merged.append(None)
                continue
            merged.append({k: torch.cat([sc[i][k] for sc in per_scene], 0) for k in per_scene[0][i]})
        return merged

    @staticmethod
    def _metric_flags(views) -> List[bool]:
        out = []
        for v in views:
            m = v.get("is_metric_scale")
            out.append(True if m is None else bool(torch.as_tensor(m).reshape(-1)[0].item()))
        return out

    def _geo_inputs(self, views, plan, metric, use_calibration=True, use_depth=True, use_pose=True,
                    use_depth_scale=True, use_pose_scale=True):
        """GeoInputs for this rank's views with infer()'s deterministic masks (model.py:1292-1438, 2154-2197)."""
        from .engine import GeoInputs

        if not (use_calibration or use_depth or use_pose):
            return None
        V = len(views)
        local = list(plan.local_views) if plan is not None else list(range(V))
        s0 = local[0]
        H, W = views[0]["img"].shape[-2:]
        dev = self._device
        g = GeoInputs(local_start=s0)
        f32 = torch.float32
        if use_calibration and any("ray_directions_cam" in views[v] for v in local):
            g.ray_views = [i for i, v in enumerate(local) if "ray_directions_cam" in views[v]]
            g.rays = torch.cat([views[v]["ray_directions_cam"].to(dev, f32) if "ray_directions_cam" in views[v]
                                else torch.zeros(1, H, W, 3, device=dev, dtype=f32) for v in local], 0).contiguous()
        if use_depth and any("depth_along_ray" in views[v] for v in local):
            g.depth_views = [i for i, v in enumerate(local) if "depth_along_ray" in views[v]]
            g.depth = torch.cat([views[v]["depth_along_ray"].to(dev, f32).reshape(1, H, W)
                                 if "depth_along_ray" in views[v] else torch.zeros(1, H, W, device=dev, dtype=f32)
                                 for v in local], 0).contiguous()
            g.depth_metric = [bool(metric[v] and use_depth_scale) for v in local]
        has_pose = [("camera_pose_quats" in v and "camera_pose_trans" in v) for v in views]
        if use_pose and any(has_pose):
            g.cam_mask = has_pose
            g.pose_metric = [bool(metric[v] and use_pose_scale) for v in range(V)]
            ident_q = torch.tensor([[0.0, 0.0, 0.0, 1.0]], device=dev, dtype=f32)
            g.cam_quats = torch.cat([views[v]["camera_pose_quats"].to(dev, f32).reshape(1, 4) if has_pose[v]
                                     else ident_q for v in range(V)], 0)
            g.cam_trans = torch.cat([views[v]["camera_pose_trans"].to(dev, f32).reshape(1, 3) if has_pose[v]
                                     else torch.zeros(1, 3, device=dev, dtype=f32) for v in range(V)], 0)
        return None if g.empty() else g

    def _geo_inputs_scenes(self, views, B, metrics, plan=None, **use):
        """GeoInputs of B batched scenes: each scene's inputs as _geo_inputs builds them (its own metric flags, its
        own camera normalisation frame), concatenated scene-major with GeoInputs.scenes = B — dense inputs over this
        rank's images (image b*n + i, n = local views per scene; n = V unsharded), camera arrays over every view
        (b*V + v); scenes without an input kind get the reference's zero / identity fill and a cleared mask.
        metrics[b]: scene b's per-view is_metric_scale flags (read on the host before the inputs moved to the
        device)."""
        from .engine import GeoInputs

        per = [self._geo_inputs(self._scene_views(views, b, B), plan, metrics[b], **use) for b in range(B)]
        if all(g is None for g in per):
            return None
        V = len(views)
        n = V if plan is None else len(plan.local_views)
        s0 = 0 if plan is None else plan.local_views[0]
        H, W = views[0]["img"].shape[-2:]
        dev, f32 = self._device, torch.float32
        g = GeoInputs(local_start=s0, scenes=B)
        if any(p is not None and p.ray_views for p in per):
            g.rays = torch.cat([p.rays if p is not None and p.ray_views else torch.zeros(n, H, W, 3, device=dev, dtype=f32)
                                for p in per], 0).contiguous()
            g.ray_views = [b * n + i for b, p in enumerate(per) if p is not None for i in p.ray_views]
        if any(p is not None and p.depth_views for p in per):
            g.depth = torch.cat([p.depth if p is not None and p.depth_views else torch.zeros(n, H, W, device=dev, dtype=f32)
                                 for p in per], 0).contiguous()
            g.depth_views = [b * n + i for b, p in enumerate(per) if p is not None for i in p.depth_views]
            g.depth_metric = [bool(p is not None and p.depth_views and p.depth_metric[i]) for p in per for i in range(n)]
        if any(p is not None and any(p.cam_mask) for p in per):
            ident_q = torch.tensor([[0.0, 0.0, 0.0, 1.0]], device=dev, dtype=f32).expand(V, 4)
            has = [p is not None and any(p.cam_mask) for p in per]
            g.cam_quats = torch.cat([p.cam_quats if h else ident_q for p, h in zip(per, has)], 0).contiguous()
            g.cam_trans = torch.cat([p.cam_trans if h else torch.zeros(V, 3, device=dev, dtype=f32)
                                     for p, h in zip(per, has)], 0).contiguous()
            g.cam_mask = [bool(h and p.cam_mask[i]) for p, h in zip(per, has) for i in range(V)]
            g.pose_metric = [bool(h and p.pose_metric[i]) for p, h in zip(per, has) for i in range(V)]
        return None if g.empty() else g

    def forward(self, views: List[Dict[str, Any]], memory_efficient_inference: bool = False,
                precision: Optional[str] = None) -> List[Dict[str, torch.Tensor]]:
        """Raw per-view outputs of model.py:1657-2152 (pts3d, pts3d_cam, ray_directions, depth_along_ray,
        cam_trans, cam_quats, metric_scaling_factor, conf, non_ambiguous_mask, non_ambiguous_mask_logits).
        Views are in the preprocessed form (ray_directions_cam, depth_along_ray, camera_pose_quats/trans,
        is_metric_scale); every provided geometric input is used (infer()'s deterministic masks)."""
        B = self._check_views(views)
        if B > 1 and not self._batchable(views):
            return self._merge_scenes([self.forward(self._scene_views(views, b, B), memory_efficient_inference,
                                                    precision) for b in range(B)])
        dnt = views[0].get("data_norm_type", ["dinov2"])
        if (dnt[0] if isinstance(dnt, (list, tuple)) else dnt) != "dinov2":
            raise AssertionError(f"Input data norm type {dnt} does not match encoder norm type dinov2")
        local, plan = self._local_views(views, B)
        geo = self._geo_inputs(views, plan, self._metric_flags(views)) if B == 1 else \
            self._geo_inputs_scenes(views, B, [self._metric_flags(self._scene_views(views, b, B)) for b in range(B)],
                                    plan)
        imgs = self._scene_major(torch.cat([v["img"] for v in local], 0).to(self._device, torch.float32), B)
        eng = self.engine(precision)
        raw = self._run_engine(eng, imgs, plan, geo, self._dpt_chunk(memory_efficient_inference), scenes=B)
        if self._await_faults(plan, eng):  # binary16 range left: this call again with the fp32-exact heads
            eng = self._range_fallback(precision)
            raw = self._run_engine(eng, imgs, plan, geo, self._dpt_chunk(memory_efficient_inference), scenes=B)
            self._await_faults(plan)
        return self._finish(raw, plan, len(views), with_post=False, scenes=B)

    # entries a view may carry and still run in a batched-scene engine call: images and every geometric input
    # (raw as infer() takes them, and preprocessed as forward() takes them)
    _BATCHABLE_KEYS = frozenset(("img", "data_norm_type", "instance", "idx", "true_shape", "is_metric_scale", "label",
                                 "intrinsics", "ray_directions", "depth_z", "camera_poses", "ray_directions_cam",
                                 "depth_along_ray", "camera_pose_quats", "camera_pose_trans"))

    def _batchable(self, views) -> bool:
        """B > 1 scenes run as ONE engine call (encoder, geometric encoders, frame layers and heads over all B x V
        images; the global layers and the camera-translation normalisation per scene; the reference's batched
        forward, model.py:687-721).  On a view-sharded model every rank holds its views of each scene
        (ShardPlan.scenes)."""
        return all(set(v.keys()) <= self._BATCHABLE_KEYS for v in views)

    @staticmethod
    def _scene_major(imgs, B: int):
        """View-major (V*B, ...) images (the per-view (B, ...) tensors concatenated) -> scene-major (B*V, ...)."""
        if B == 1:
            return imgs
        V = imgs.shape[0] // B
        return imgs.view(V, B, *imgs.shape[1:]).transpose(0, 1).reshape(imgs.shape).contiguous()

    _MAX_GRAPHS = 4

    def _view_pe_rows(self, num_views: int) -> Optional[torch.Tensor]:
        """View-PE table rows of this forward (None when only the reference view is encoded): 0 for the reference
        view, then torch.randint(1, rows, (V-1,)) from the global CPU generator, the same draw the reference makes
        per forward (alternating_attention_transformer.py:608-611, global_attention_transformer.py:551-554), or
        1..V-1 without random indices."""
        if not self.info.nonref_pe:
            return None
        if self.info.rand_idx:
            rest = torch.randint(low=1, high=self.info.pe_rows, size=(num_views - 1,))
        else:
            if num_views > self.info.pe_rows:
                raise ValueError(f"{num_views} views exceed the {self.info.pe_rows}-row view positional table")
            rest = torch.arange(1, num_views)
        return torch.cat([torch.zeros(1, dtype=torch.int64), rest.to(torch.int64)]).to(self._device)

    def _run_engine(self, eng, imgs, plan, geo, dpt_chunk, scenes: int = 1):
        """MapaEngine.run, replayed from a captured HIP graph when the call is graph-safe: no
        chunked dense head, no per-launch kernel timing, not in the serialize debug mode (every launch checked,
        nat.SERIALIZE), and either one device or a view shard whose communicator enqueues its collectives on the
        device (DistComm over RCCL: the K/V all-gathers and the scale-token broadcast are captured with the
        kernels, forking to and joining from the communicator's stream).  The graph is keyed on the image batch
        shape, precision, shard plan and the geometric inputs' structure (GeoInputs.signature: which views carry
        rays / depth / poses, the metric flags); images, view-PE rows and geometric tensors are copied into its
        static buffers and outputs cloned out of it, so results never alias a later call's."""
        pe_idx = self._view_pe_rows(plan.num_views if plan is not None else imgs.shape[0] // scenes)
        shard_ok = plan is None or (self._shard_graphs and getattr(self._comm, "graph_safe", False))
        if (not self.hip_graphs or not shard_ok or dpt_chunk is not None
                or nat._timing is not None or nat.SERIALIZE or imgs.device.type != "cuda"):
            return eng.run(imgs, shard=plan, comm=self._comm, geo=geo, dpt_chunk=dpt_chunk, pe_idx=pe_idx,
                           scenes=scenes, fault=self._arm_fault())
        pkey = None if plan is None else (plan.world, plan.rank, tuple(plan.counts), force_collectives(),
                                          force_overlap(), os.environ.get("MAPA_KV_OVERLAP", "1"))
        key = (eng.precision, eng.heads, tuple(imgs.shape), imgs.device.index, scenes,
               None if geo is None else geo.signature(), pkey)
        comm = self._comm if plan is not None else None
        with torch.inference_mode():  # static buffers are inference tensors whichever mode the first call ran in
            entry = self._graphs.get(key)
            if entry is None:
                static_in = imgs.clone()
                static_pe = None if pe_idx is None else pe_idx.clone()  # refreshed before every replay
                static_geo = None if geo is None else geo.static_copy()  # geometric inputs: likewise
                side = torch.cuda.Stream(imgs.device)
                side.wait_stream(torch.cuda.current_stream(imgs.device))
                with torch.cuda.stream(side):  # eager warm-up: lazy packing, pos-embed caches
                    eng.run(static_in, shard=plan, comm=comm, geo=static_geo, pe_idx=static_pe, scenes=scenes,
                            fault=self._arm_fault())
                    try:
                        self._await_local_fault()
                    except nat.DeviceFault as e:
                        # binary16 range left in the warm-up: capture anyway (every rank captures the same
                        # collectives); the replay below reports it again and the caller re-runs with the fp32-exact
                        # heads (_await_faults -> _range_fallback)
                        if not (e.range_only and eng.hsplit and eng.hfmt in ("f16", "f16x2")):
                            raise
                torch.cuda.current_stream(imgs.device).wait_stream(side)
                graph = torch.cuda.CUDAGraph()
                gslot = nat.FaultSlot()  # the graph's own publish slot (its address is baked into the graph)
                # captured on the warm-up stream: the per-stream GEMM / attention workspaces made in the warm-up
                # are the ones the graph uses (no allocation or zero-fill inside the capture).  With a shard the
                # capture is thread-local: the communicator's watchdog thread keeps querying its events meanwhile
                mode = "global" if plan is None else "thread_local"
                if plan is None:
                    with torch.cuda.graph(graph, stream=side, capture_error_mode=mode):
                        static_out = eng.run(static_in, shard=plan, comm=comm, geo=static_geo, pe_idx=static_pe,
                                             scenes=scenes, fault=gslot)
                else:
                    # every rank captures the same collectives in the same order, so a capture that fails on one
                    # rank fails on all; the ranks still agree (one eager all-reduce) before any replays, and fall
                    # back to the eager sharded path together, whose collectives match a replay's one for one
                    err = None
                    try:
                        with torch.cuda.graph(graph, stream=side, capture_error_mode=mode):
                            static_out = eng.run(static_in, shard=plan, comm=comm, geo=static_geo, pe_idx=static_pe,
                                                 scenes=scenes, fault=gslot)
                    except Exception as e:  # noqa: BLE001 -- any capture failure: agree, then run eager
                        err = e
                        if os.environ.get("MAPA_GRAPH_DEBUG"):
                            import traceback
                            traceback.print_exc()
                            raise
                    if not self._comm.all_agree(err is None, imgs.device):
                        warnings.warn(f"sharded HIP-graph capture failed ({err or 'on another rank'}); "
                                      "running the sharded path eagerly on the process group")
                        self._shard_graphs = False
                        self.shard_graph_fallback = f"sharded HIP-graph capture failed: {err or 'on another rank'}"
                        from ...parallel import DistComm, RcclComm

                        if isinstance(self._comm, RcclComm):  # an aborted capture may leave its RCCL state unusable
                            old, self._comm = self._comm, DistComm(self._comm.group)
                            old.close(abort=True)
                        return eng.run(imgs, shard=plan, comm=self._comm, geo=geo, pe_idx=pe_idx, scenes=scenes,
                                       fault=self._arm_fault())
                # the side stream is kept with the graph: its handle keys the per-stream workspaces the graph
                # captured (_native._WS/_AWS), so it must not be destroyed and its handle reused while the graph lives
                entry = (graph, static_in, static_out, static_pe, side, gslot, static_geo)
                self._graphs[key] = entry
                while len(self._graphs) > self._MAX_GRAPHS:
                    self._graphs.popitem(last=False)
            else:
                self._graphs.move_to_end(key)
            graph, static_in, static_out, static_pe, _side, gslot, static_geo = entry
            static_in.copy_(imgs)
            if static_pe is not None:
                static_pe.copy_(pe_idx)
            if static_geo is not None:
                geo.refresh_into(static_geo)
            gslot.arm()
            self._fault_state().pending = gslot
            graph.replay()
        return {k: v.clone() for k, v in static_out.items()}

    # ----------------------------------------------------------------------------------- device fault channel
    def _fault_state(self):
        """Per-thread fault-channel state (the in-thread sharding tests drive one model from several rank threads):
        .eager = this thread's slot for eager runs, .pending = the slot this thread's current call waits on."""
        st = self.__dict__.get("_fault_tls")
        if st is None:
            import threading

            st = self.__dict__.setdefault("_fault_tls", threading.local())
        if not hasattr(st, "pending"):
            st.eager, st.pending = None, None
        return st

    def _arm_fault(self):
        """This thread's eager fault slot, armed; the run publishes the device fault word into it after the
        transformer (engine.run), and the caller checks it before returning (_await_faults)."""
        st = self._fault_state()
        if st.eager is None:
            st.eager = nat.FaultSlot()
        st.eager.arm()
        st.pending = st.eager
        return st.eager

    def _await_local_fault(self):
        st = self._fault_state()
        slot, st.pending = st.pending, None
        if slot is not None:
            slot.wait()

    # binary16 range fallbacks taken (MAPA_FAULT_F16_RANGE under the TF32-equivalent heads; bench.py reports it)
    range_fallbacks = 0

    def _range_fallback(self, precision):
        """The engine a call re-runs on after its TF32-equivalent (binary16) heads or geometric encoders left
        binary16's range: the fp32-exact split-precision heads (head_precision='fp32'), whose operands cover fp32's
        range as the reference's TF32 does (model.py:89-93, 1774).  Counted in range_fallbacks; warned once."""
        MapAnything.range_fallbacks += 1
        if MapAnything.range_fallbacks == 1:
            warnings.warn("a binary16 head operand left binary16's range (MAPA_FAULT_F16_RANGE): the call was re-run "
                          "with the fp32-exact heads (head_precision='fp32'); later calls do the same when needed")
        return self.engine(precision, heads="fp32")

    def _comm_failed(self, comm, why: str):
        """The communicator was aborted (a hung or failed collective): graphs captured against it hold its freed RCCL
        state, so they are dropped and the model refuses sharded calls until enable_view_sharding() installs a new
        communicator (a replay on an aborted communicator faults instead of raising)."""
        for k in [k for k in self._graphs if k[-1] is not None]:
            del self._graphs[k]
        if hasattr(comm, "graph_safe"):
            comm.graph_safe = False
        self._shard_graphs = False
        self.shard_graph_fallback = f"communicator aborted: {why}"
        self._comm_dead = why

    def _await_faults(self, plan, eng=None) -> bool:
        """Wait for this call's fault publish (the GPU is past the transformer then and still has the heads queued,
        so the wait costs no GPU time) and raise NativeError if a kernel set the device fault word — a LayerNorm-
        fused band barrier that timed out (include/mapa.h fault channel): the outputs are then never returned.
        Returns True instead when the only fault is MAPA_FAULT_F16_RANGE and `eng` runs binary16 ("tf32") heads /
        geometric encoders: the caller re-runs the call with the fp32-exact heads (_range_fallback).  A sharded
        model agrees across ranks first — whenever it gathers outputs or a range fallback is possible — so every rank
        raises, or re-runs its collectives, together instead of one rank leaving the others in a collective."""
        err = None
        st = self._fault_state()
        slot, st.pending = st.pending, None
        if slot is not None and os.environ.get("MAPA_FAULT_WAIT", "1") == "0":  # A/B switch: publish, never wait
            slot.armed = False
            slot = None
        comm = self._comm if plan is not None else None
        if slot is not None:
            from ...parallel import CommError

            try:
                if comm is None:
                    slot.wait()
                else:  # sharded: a hung collective never lets the forward reach its publish
                    slot.wait(timeout_s=comm_timeout().total_seconds(), poll=getattr(comm, "check_async", None))
            except nat.FaultTimeout as e:
                if comm is None:
                    raise
                if hasattr(comm, "abort"):
                    comm.abort()  # RCCL's kernels stop on the abort flag; the stream can drain
                self._comm_failed(comm, f"rank {plan.rank}: forward not complete ({e})")
                raise CommError(f"sharded forward on rank {plan.rank} did not complete: {e} (RCCL communicator "
                                "aborted)") from e
            except CommError as e:  # check_async: the communicator reported an error (and was aborted)
                self._comm_failed(comm, str(e))
                raise
            except nat.NativeError as e:
                err = e
        range_ok = eng is not None and eng.hsplit and eng.hfmt in ("f16", "f16x2")
        retry = range_ok and isinstance(err, nat.DeviceFault) and err.range_only
        if plan is not None and plan.world > 1 and hasattr(self._comm, "all_agree") and \
                (self._gather is not None or range_ok):
            # host-side agreement where the communicator has one (a gloo group: the GPU keeps running the heads)
            agree = getattr(self._comm, "all_agree_host", None) or (lambda ok: self._comm.all_agree(ok, self._device))
            if agree(err is None):
                return False
            if range_ok and agree(err is None or retry):
                err = None
                return True  # every rank re-runs (their collectives pair up again)
            raise err or nat.NativeError("a device fault on another rank (include/mapa.h fault channel)")
        if err is not None and not retry:
            raise err
        err = None  # (the exception's traceback holds this frame: drop the cycle so the fault slot is freed now)
        return retry

    @torch.inference_mode()
    def infer(self, views: List[Dict[str, Any]], memory_efficient_inference: bool = False, use_amp: bool = True,
              amp_dtype: str = "bf16", apply_mask: bool = True, mask_edges: bool = True,
              edge_normal_threshold: float = 5.0, edge_depth_threshold: float = 0.03,
              apply_confidence_mask: bool = False, confidence_percentile: float = 10,
              ignore_calibration_inputs: bool = False, ignore_depth_inputs: bool = False,
              ignore_pose_inputs: bool = False, ignore_depth_scale_inputs: bool = False,
              ignore_pose_scale_inputs: bool = False) -> List[Dict[str, torch.Tensor]]:
        """model.py:2206-2355."""
        # autocast recipe (model.py:2287-2302): bf16 or fp16 operands for the encoder and the transformer; the
        # geometric encoders and the heads fp32 as the reference runs them (autocast disabled, model.py:1377 / 1774)
        if use_amp and amp_dtype in ("bf16", "fp16"):
            precision = amp_dtype
        else:
            if use_amp and amp_dtype not in ("bf16", "fp16", "fp32"):
                warnings.warn(f"unknown amp_dtype {amp_dtype!r}: running fp32")
            precision = "fp32"
        validated = validate_input_views_for_inference(views)
        B = self._check_views(validated)
        if B > 1 and not self._batchable(validated):
            # scene by scene (module docstring), outputs concatenated per view as the reference returns them
            kw = dict(memory_efficient_inference=memory_efficient_inference, use_amp=use_amp, amp_dtype=amp_dtype,
                      apply_mask=apply_mask, mask_edges=mask_edges, edge_normal_threshold=edge_normal_threshold,
                      edge_depth_threshold=edge_depth_threshold, apply_confidence_mask=apply_confidence_mask,
                      confidence_percentile=confidence_percentile, ignore_calibration_inputs=ignore_calibration_inputs,
                      ignore_depth_inputs=ignore_depth_inputs, ignore_pose_inputs=ignore_pose_inputs,
                      ignore_depth_scale_inputs=ignore_depth_scale_inputs,
                      ignore_pose_scale_inputs=ignore_pose_scale_inputs)
            return self._merge_scenes([self.infer(self._scene_views(validated, b, B), **kw) for b in range(B)])
        # host-side flags read before the H2D copies (per scene when B > 1)
        metric = self._metric_flags(validated) if B == 1 else \
            [self._metric_flags(self._scene_views(validated, b, B)) for b in range(B)]
        for v in validated:
            for k in list(v.keys()):
                if k in ("instance", "idx", "true_shape", "data_norm_type"):
                    continue
                if isinstance(v[k], torch.Tensor):
                    v[k] = v[k].to(self._device, non_blocking=True)
                elif isinstance(v[k], tuple):
                    v[k] = tuple(x.to(self._device, non_blocking=True) if isinstance(x, torch.Tensor) else x
                                 for x in v[k])
        processed = preprocess_input_views_for_inference(validated)
        local, plan = self._local_views(processed, B)
        use = dict(use_calibration=not ignore_calibration_inputs, use_depth=not ignore_depth_inputs,
                   use_pose=not ignore_pose_inputs, use_depth_scale=not ignore_depth_scale_inputs,
                   use_pose_scale=not ignore_pose_scale_inputs)
        if B == 1:
            geo = self._geo_inputs(processed, plan, metric, **use)
        else:
            geo = self._geo_inputs_scenes(processed, B, metric, plan, **use)
        imgs = self._scene_major(torch.cat([v["img"] for v in local], 0).to(self._device, torch.float32), B)
        eng = self.engine(precision)

        def run(eng):
            raw = self._run_engine(eng, imgs, plan, geo, self._dpt_chunk(memory_efficient_inference), scenes=B)
            return postprocess_outputs(raw, imgs, eng.w.norm_mean, eng.w.norm_std, apply_mask=apply_mask,
                                       mask_edges=mask_edges, edge_normal_threshold=edge_normal_threshold,
                                       edge_depth_threshold=edge_depth_threshold,
                                       apply_confidence_mask=apply_confidence_mask,
                                       confidence_percentile=confidence_percentile)
        post = run(eng)
        if self._await_faults(plan, eng):  # binary16 range left: this call again with the fp32-exact heads
            post = run(self._range_fallback(precision))
            self._await_faults(plan)
        return self._finish(post, plan, len(views), with_post=True, scenes=B)

    def _dpt_chunk(self, memory_efficient: bool):
        """Views per dense-head pass.  memory_efficient_inference mirrors _compute_adaptive_minibatch_size
        (model.py:1440-1477): 95 % of free HBM over a per-view bound (the dense head's peak at 518²: ≈420 MB with
        fp32-exact split-precision heads — the 518² split operand of the last conv plus its fp32 output — ≈320 MB
        with bf16 heads; the reference's is 680 MB); otherwise every view in one pass."""
        if not memory_efficient:
            return None
        free = torch.cuda.mem_get_info(self._device)[0]
        per_view = 320 if self.heads_for(self.precision) == "bf16" else 420
        return max(1, int(0.95 * free / (per_view * 1024 * 1024)))

    def _local_views(self, views, scenes: int = 1):
        if self._comm is None:
            return views, None
        if getattr(self, "_comm_dead", None):
            from ...parallel import CommError

            raise CommError(f"the view-sharding communicator was aborted ({self._comm_dead}); call "
                            "enable_view_sharding() again")
        from ...parallel import ShardPlan

        H, W = views[0]["img"].shape[-2:]
        plan = ShardPlan(len(views), self._comm.world, self._comm.rank, (H // 14) * (W // 14), scenes)
        return [views[i] for i in plan.local_views], plan

    def _finish(self, batched, plan, V, with_post, scenes: int = 1):
        """Batched view-major outputs of this rank -> the reference's per-view list (gathered across ranks when
        enable_view_sharding(gather_outputs=...) asks for it).  scenes > 1: scene-major outputs of B batched scenes
        -> per view (B, ...) tensors."""
        if plan is None:
            return split_views(batched, V, with_post, scenes)
        B = scenes
        if self._gather is not None and plan.world > 1:
            dst = 0 if self._gather == "rank0" else None
            counts = [B * c for c in plan.counts]
            # gathered rows are rank-major ([rank][scene][view]); scene-major order [scene][global view]
            order = None if B == 1 else torch.tensor(
                [sum(counts[:r]) + b * plan.counts[r] + i for b in range(B) for r in range(plan.world)
                 for i in range(plan.counts[r])])
            full = {}
            for k, t in batched.items():
                # metric_scaling_factor is already the same on every rank (rank 0's scale token, engine.aat)
                if k == "metric_scaling_factor":
                    full[k] = t
                    continue
                g = self._comm.gather_views(t, counts, dst)
                full[k] = g if g is None or order is None else g.index_select(0, order.to(g.device))
            if dst is None or plan.rank == dst:
                return split_views(full, V, with_post, scenes)
        local_out = split_views(batched, len(plan.local_views), with_post, scenes)
        out = [None] * V
        for i, v in enumerate(plan.local_views):
            out[v] = local_out[i]
        return out

    __call__ = forward


def split_views(out: Dict[str, torch.Tensor], V: int, with_post: bool, scenes: int = 1) -> List[Dict[str, torch.Tensor]]:
    """Batched outputs -> the reference's list of per-view dicts: B = 1 as views of the view-major rows (no copies);
    B = scenes > 1 from scene-major rows (image b*V + v) gathered into (B, ...) per view."""
    res = []
    B = scenes
    for i in range(V):
        d = {}
        sel = None if B == 1 else torch.arange(B, device=next(iter(out.values())).device) * V + i
        for k, t in out.items():
            if k == "metric_scaling_factor":  # one row per scene, shared by its views
                d[k] = t
                continue
            x = t[i:i + 1] if sel is None else t.index_select(0, sel)
            if k == "non_ambiguous_mask":
                d[k] = x.bool()
            elif k == "mask":
                d[k] = x.bool().unsqueeze(-1)
            else:
                d[k] = x
        if "pts3d_cam" in d:
            d["depth_z"] = d["pts3d_cam"][..., 2:3]
        res.append(d)
    return res


def _strip_comments(txt: str) -> str:
    import re

    return re.sub(r"//[^\n]*", "", txt)

"""Host-side logic: state-dict layout vs the reference, synthetic checkpoint determinism, input validation."""

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def test_state_dict_layout_matches_reference():
    from mapanything.models.mapanything.spec import canonical_spec, full_spec

    ref = json.load(open(os.path.join(GOLDEN, "ref_state_dict_spec.json")))
    mine = dict(full_spec())
    assert len(ref) == len(mine) == 880
    for k, shape in ref:
        assert tuple(mine[k]) == tuple(shape), k
    assert sum(int(np.prod(s)) for _, s in canonical_spec()) == 563336150


def test_synthetic_generator_is_deterministic_and_scaled():
    from mapanything.utils.synthetic import named_uniform, splitmix_uniform, tensor_init

    a = named_uniform("x.weight", (64, 32), -1, 1)
    b = named_uniform("x.weight", (64, 32), -1, 1)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, named_uniform("y.weight", (64, 32), -1, 1))
    u = splitmix_uniform(12345, 100000)
    assert u.min() >= 0 and u.max() < 1 and abs(u.mean() - 0.5) < 0.01
    w = tensor_init("info_sharing.self_attention_blocks.0.mlp.fc1.weight", (3072, 768))
    assert abs(np.abs(w).max() - np.sqrt(3 / 768)) < 1e-3
    pe = tensor_init("info_sharing.view_pos_table", (1, 768))
    assert np.array_equal(pe[0, 0::2], np.zeros(384, np.float32)) and np.array_equal(pe[0, 1::2], np.ones(384))


def test_validation_errors_match_reference_rules():
    from mapanything.utils.inference import validate_input_views_for_inference as val

    img = torch.zeros(1, 3, 28, 28)
    with pytest.raises(ValueError, match="At least one view"):
        val([])
    with pytest.raises(ValueError, match="missing required keys"):
        val([{"img": img}])
    with pytest.raises(ValueError, match="conflicting keys"):
        val([{"img": img, "data_norm_type": ["dinov2"], "intrinsics": 1, "ray_directions": 2}])
    with pytest.raises(ValueError, match="depth constraint"):
        val([{"img": img, "data_norm_type": ["dinov2"], "depth_z": 1}])
    with pytest.raises(ValueError, match="Camera pose constraint"):
        val([{"img": img, "data_norm_type": ["dinov2"]},
             {"img": img, "data_norm_type": ["dinov2"], "camera_poses": 1}])
    with pytest.raises(ValueError, match="First View"):
        val([{"data_norm_type": ["dinov2"], "intrinsics": 1, "camera_poses": 1}])
    ok = [{"img": img, "data_norm_type": ["dinov2"]}]
    assert val(ok) is ok


@pytest.mark.gpu
def test_preprocess_matches_oracle_restatement():
    """Per-pixel preprocessing runs in the mapa_view_rays kernel (GPU); compared with the oracle's CPU restatement."""
    from mapanything.utils.inference import preprocess_input_views_for_inference
    from oracle.mapa_oracle import preprocess_views

    K = torch.tensor([[[30.0, 0, 14.0], [0, 31.0, 13.5], [0, 0, 1]]])
    d = torch.rand(1, 28, 28, generator=torch.Generator().manual_seed(0)) * 5
    q = torch.tensor([[0.1, 0.2, 0.3, 0.9]])
    q = q / q.norm()
    views = [{"img": torch.zeros(1, 3, 28, 28), "data_norm_type": ["dinov2"], "intrinsics": K, "depth_z": d,
              "camera_poses": (q, torch.tensor([[1.0, 2.0, 3.0]]))}]
    gpu_views = [{k: (v.cuda() if torch.is_tensor(v) else tuple(x.cuda() for x in v) if isinstance(v, tuple) else v)
                  for k, v in view.items()} for view in views]
    a = preprocess_input_views_for_inference(gpu_views)[0]
    b = preprocess_views([dict(v) for v in views])[0]
    for k in ("ray_directions_cam", "depth_along_ray", "camera_pose_quats", "camera_pose_trans"):
        assert torch.allclose(a[k].cpu(), b[k], atol=1e-6), k
    assert bool(a["is_metric_scale"].all())


def test_config_guard_rejects_other_architectures():
    from mapanything.models import MapAnything
    from tests_helpers import released_config

    cfg = released_config()
    m = MapAnything(**cfg)
    assert m.class_init_args["name"] == "mapanything"
    cfg["pred_head_config"] = dict(cfg["pred_head_config"], type="linear")
    with pytest.raises(ValueError, match="unsupported"):
        MapAnything(**cfg)


def test_module_surface_is_exposed():
    """The sub-modules the reference's forward calls (model.py:168-634) exist under the same attribute names and
    take the uniception dataclasses (tests/test_gpu_modules.py runs them)."""
    from mapanything.models import MapAnything
    from tests_helpers import released_config
    from uniception.models.encoders import ViTEncoderInput, ViTEncoderOutput  # noqa: F401
    from uniception.models.info_sharing import MultiViewTransformerInput, MultiViewTransformerOutput  # noqa: F401
    from uniception.models.prediction_heads import (AdaptorInput, DPTFeatureInput, PixelTaskOutput,  # noqa: F401
                                                    PredictionHeadInput, PredictionHeadLayeredInput,
                                                    PredictionHeadTokenInput, SummaryTaskOutput)

    m = MapAnything(**released_config())
    for name in ("encoder", "info_sharing", "dpt_feature_head", "dpt_regressor_head", "dense_head", "dense_adaptor",
                 "pose_head", "pose_adaptor", "scale_head", "scale_adaptor", "fusion_norm_layer"):
        assert callable(getattr(m, name)), name
    assert m.encoder is m.encoder and m.info_sharing.indices == (11, 17)


def _released_model(**kw):
    from mapanything.models import MapAnything
    from tests_helpers import released_config

    return MapAnything(**released_config(), **kw)


@pytest.mark.parametrize("layout", ["all_880_keys", "deduplicated"])
def test_from_pretrained_local_safetensors(tmp_path, layout):
    """MapAnything.from_pretrained(local_dir) reads config.json + model.safetensors written under the reference's
    state-dict names (model.py:17, 96): either every one of the 880 keys (aliases included, as nn.Module's
    state_dict lists them) or one name per shared tensor (safetensors' save_model de-duplication).  The loaded
    weights equal the synthetic checkpoint exactly."""
    from safetensors.numpy import save_file

    from mapanything.models import MapAnything
    from mapanything.models.mapanything.spec import aliases
    from tests_helpers import released_config

    src = _released_model().load_synthetic_weights()
    sd = src.state_dict()
    ref_names = [k for k, _ in json.load(open(os.path.join(GOLDEN, "ref_state_dict_spec.json")))]
    assert list(sd.keys()) == ref_names or sorted(sd.keys()) == sorted(ref_names)
    if layout == "deduplicated":
        al = aliases()
        sd = {k: v for k, v in sd.items() if k not in al}
    save_file({k: v.numpy().copy() for k, v in sd.items()}, str(tmp_path / "model.safetensors"))
    with open(tmp_path / "config.json", "w") as f:
        json.dump(released_config(), f)
    m = MapAnything.from_pretrained(str(tmp_path), head_precision="bf16")
    assert m.head_precision == "bf16"
    assert set(m._sd) == set(src._sd)
    for k in src._sd:
        assert np.array_equal(m._sd[k], src._sd[k]), k
    # state_dict aliases share storage with their canonical tensor, as in the reference
    full = m.state_dict()
    assert full["dense_head.0.scratch.layer1_rn.weight"].data_ptr() == \
        full["dpt_feature_head.scratch.layer1_rn.weight"].data_ptr()
    assert len(list(m.parameters())) == len(src._sd)


def test_save_pretrained_round_trip(tmp_path):
    from mapanything.models import MapAnything

    src = _released_model().load_synthetic_weights()
    src.save_pretrained(str(tmp_path))
    m = MapAnything.from_pretrained(str(tmp_path))
    for k in src._sd:
        assert np.array_equal(m._sd[k], src._sd[k]), k
    with pytest.raises(FileNotFoundError):
        MapAnything.from_pretrained(str(tmp_path / "missing"))


def test_batched_scene_layout_round_trip():
    """B scenes x V views: the per-view (B, ...) image tensors concatenated view-major -> scene-major engine rows
    (image b*V + v) -> split_views gives each view back its (B, ...) rows in scene order (reference model.py:687-721
    batches scenes along dim 0 of every view)."""
    from mapanything.models.mapanything.model import MapAnything, split_views

    V, B = 3, 2
    per_view = [torch.arange(B * 4, dtype=torch.float32).view(B, 1, 2, 2) + 100 * v for v in range(V)]
    rows = MapAnything._scene_major(torch.cat(per_view, 0), B)
    for b in range(B):
        for v in range(V):
            assert torch.equal(rows[b * V + v], per_view[v][b])
    msf = torch.tensor([[1.5], [2.5]])
    out = split_views({"pts3d": rows.permute(0, 2, 3, 1).expand(-1, -1, -1, 3).contiguous(),
                       "non_ambiguous_mask": (rows[:, 0] > 102).to(torch.uint8), "metric_scaling_factor": msf},
                      V, with_post=False, scenes=B)
    assert len(out) == V
    for v in range(V):
        assert out[v]["pts3d"].shape == (B, 2, 2, 3)
        assert torch.equal(out[v]["pts3d"][..., 0], per_view[v][:, 0])
        assert out[v]["non_ambiguous_mask"].dtype == torch.bool
        assert torch.equal(out[v]["non_ambiguous_mask"], per_view[v][:, 0] > 102)
        assert torch.equal(out[v]["metric_scaling_factor"], msf)
    assert torch.equal(MapAnything._scene_major(rows, 1), rows)


def test_aborted_communicator_drops_sharded_graphs_and_refuses_sharded_calls():
    """after a sharded call's communicator is aborted (a hung or failed collective), the HIP
    graphs captured against it hold its freed RCCL state.  MapAnything._comm_failed drops exactly those graphs (the
    unsharded ones stay), marks the communicator and the model unfit for sharded capture, and every later sharded
    call raises CommError — no replay on the dead communicator — until enable_view_sharding() installs a new one,
    which allows sharded graphs again."""
    import torch

    from mapanything.parallel import CommError

    class FakeComm:
        world, rank, graph_safe = 2, 0, True

        def __init__(self):
            self.closed = False

        def close(self, abort=False):
            self.closed = True

    m = _released_model()
    c1 = FakeComm()
    m.enable_view_sharding(comm=c1)
    assert m._shard_graphs
    m._graphs[("bf16", "tf32", (4, 3, 518, 518), 0, 1, None, None)] = "unsharded graph"
    m._graphs[("bf16", "tf32", (4, 3, 518, 518), 0, 1, None, (2, 0, (4, 4), False, False, "1"))] = "sharded graph"
    m._comm_failed(c1, "rank 0: forward not complete (test)")
    assert list(m._graphs.values()) == ["unsharded graph"]
    assert not c1.graph_safe and not m._shard_graphs
    assert m.shard_graph_fallback.startswith("communicator aborted")
    views = [{"img": torch.zeros(1, 3, 518, 518)} for _ in range(8)]
    with pytest.raises(CommError, match="enable_view_sharding"):
        m._local_views(views)
    c2 = FakeComm()
    m.enable_view_sharding(comm=c2)
    assert c1.closed and m._comm is c2 and m._shard_graphs and m.shard_graph_fallback is None
    local, plan = m._local_views(views)
    assert plan.world == 2 and plan.rank == 0 and len(local) == 4

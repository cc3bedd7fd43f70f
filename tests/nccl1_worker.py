"""Worker of tests/test_gpu_distcomm.py::test_one_rank_rccl_sharded_graph: a real one-rank RCCL ("nccl") process
group on the test box's GPU, MAPA_FORCE_COLLECTIVES=1 so the K/V all-gathers and the scale-token broadcast run
through RCCL although the shard holds every view; the sharded forward runs eager and HIP-graph captured / replayed.
Mode "overlap" adds MAPA_FORCE_OVERLAP=1: the N > 1 production branch of every global layer — the all-gather on the
communicator's side stream forked from / joined into the capturing stream, attention over the "local" half of the
keys with LSE, attention over the "remote" half, the LSE merge.  Writes its result as JSON to argv[1]."""
import json
import os
import sys
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "map-anything_amd"))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


KEYS = ("pts3d", "conf", "depth_along_ray", "ray_directions", "cam_quats", "cam_trans", "metric_scaling_factor")


def main():
    out = sys.argv[1]
    torch.cuda.set_device(0)
    os.environ["MAPA_FORCE_COLLECTIVES"] = "1"
    os.environ["MAPA_SHARD_GRAPHS"] = "1"  # the default; set in case the caller's environment turned it off
    from mapanything.models import MapAnything
    from mapanything.parallel import init_distributed
    from mapanything.utils import synthetic
    from tests_helpers import released_config

    rank, world = init_distributed("nccl", torch.device("cuda", 0))
    assert world == 1 and dist.get_backend() == "nccl"
    from mapanything import _native as nat
    from mapanything.parallel import RcclComm

    merges = [0]
    real_merge = nat.attn_merge

    def counting_merge(*a, **k):  # counts the overlapped branch's LSE merges (eager calls and captured launches)
        merges[0] += 1
        return real_merge(*a, **k)

    nat.attn_merge = counting_merge
    V = 3
    views = [{"img": torch.from_numpy(i), "data_norm_type": ["dinov2"]}
             for i in synthetic.synthetic_images(V, 224, 224, 41)]
    # two scenes per view (batch_size_per_view 2): the batched-scene sharded global layers (one gather, per-scene
    # segment tables over the gathered slots)
    views2 = [{"img": torch.cat([v["img"], torch.from_numpy(i)], 0), "data_norm_type": ["dinov2"]}
              for v, i in zip(views, synthetic.synthetic_images(V, 224, 224, 43))]
    # two batched scenes with mixed geometric inputs (b2_224: rays / depth / poses per view; the camera inputs
    # normalised per scene and picked per local image under the capture)
    from tests_helpers import CASES, make_views

    geo2 = make_views(CASES["b2_224"])
    res = {}
    for mode in ("gather", "overlap", "scenes2", "geoscenes2"):
        os.environ["MAPA_FORCE_OVERLAP"] = "1" if mode == "overlap" else "0"
        vw = {"scenes2": views2, "geoscenes2": geo2}.get(mode, views)
        nv = len(vw)
        for prec in ("fp32", "bf16"):
            model = MapAnything(**released_config(), precision=prec).load_synthetic_weights().to("cuda")
            kw = dict(use_amp=prec == "bf16", apply_mask=False)
            single = model.infer(vw, **kw)  # unsharded (graph-replayed on one GPU)
            model.enable_view_sharding(dist.group.WORLD)
            direct = isinstance(model._comm, RcclComm)
            model.hip_graphs = False
            merges[0] = 0
            eager = model.infer(vw, **kw)
            eager_merges = merges[0]
            model.hip_graphs = True
            with warnings.catch_warnings(record=True) as caught:  # a failed capture warns and falls back to eager
                warnings.simplefilter("always")
                g1 = model.infer(vw, **kw)  # captures the sharded forward (RCCL collectives inside the graph)
            merges[0] = 0
            g2 = model.infer(vw, **kw)  # replays it (no Python-side launches)
            replay_merges = merges[0]
            torch.cuda.synchronize()
            res[f"{mode}_{prec}"] = {
                "direct_rccl": direct,
                "sharded_graph_keys": sum(1 for k in model._graphs if k[-1] is not None),
                "eager_merges": eager_merges,
                "replay_python_merges": replay_merges,
                "graph_eq_eager": all(torch.equal(a[k], b[k]) for a, b in zip(g1, eager) for k in KEYS),
                "replay_eq_eager": all(torch.equal(a[k], b[k]) for a, b in zip(g2, eager) for k in KEYS),
                "eager_eq_single": all(torch.equal(a[k], b[k]) for a, b in zip(eager, single) for k in KEYS),
                "err_vs_single": {k: max(rel(eager[v][k], single[v][k]) for v in range(nv)) for k in KEYS},
                "warnings": [str(w.message)[:500] for w in caught],
            }
            model._comm.close()
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

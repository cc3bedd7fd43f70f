"""Worker of tests/test_gpu_distcomm.py: one rank of a 2-process job on the test box's one GPU, view-sharded
through the real DistComm (torch.distributed process group, async all-gather handle, broadcast, gather).  Launched
by torch.distributed.run as child processes of the test; writes its result as JSON (argv[1] = output prefix)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "map-anything_amd"))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main():
    out_prefix = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)  # both ranks share the box's one GPU (RCCL refuses two ranks per device: gloo)
    dist.init_process_group("gloo")
    from mapanything.models import MapAnything
    from mapanything.utils import synthetic
    from tests_helpers import released_config

    V = 3
    views = [{"img": torch.from_numpy(i), "data_norm_type": ["dinov2"]}
             for i in synthetic.synthetic_images(V, 224, 224, 31)]
    model = MapAnything(**released_config(), precision="fp32").load_synthetic_weights().to("cuda")
    single = model.infer(views, use_amp=False, apply_mask=False) if rank == 0 else None
    model.enable_view_sharding(dist.group.WORLD, gather_outputs="rank0")
    res = {"rank": rank}
    for overlap in ("1", "0"):  # the overlapped async all-gather path, then gather-first
        os.environ["MAPA_KV_OVERLAP"] = overlap
        outs = model.infer(views, use_amp=False, apply_mask=False)
        torch.cuda.synchronize()
        scale = next(o for o in outs if o is not None)["metric_scaling_factor"].float().cpu()
        t = torch.tensor([float(scale.flatten()[0])])
        allt = [torch.zeros(1) for _ in range(world)]
        dist.all_gather(allt, t)
        res[f"scales_{overlap}"] = [float(x) for x in allt]
        res[f"n_views_{overlap}"] = sum(o is not None for o in outs)
        if rank == 0:
            res[f"err_{overlap}"] = {k: max(rel(outs[v][k], single[v][k]) for v in range(V))
                                     for k in ("pts3d", "conf", "cam_quats", "cam_trans", "metric_scaling_factor")}
    with open(f"{out_prefix}.{rank}.json", "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

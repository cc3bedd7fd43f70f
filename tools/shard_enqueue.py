"""Host enqueue vs GPU time of the view-sharded forward on one rank: a one-rank RCCL group with
MAPA_FORCE_COLLECTIVES=1, V views at 518x518 in the bf16 recipe; per forward: the host time until MapaEngine.run
returns (every launch enqueued), the wall time to completion, both eager and HIP-graph replayed.
  python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port P \
      tools/shard_enqueue.py [views] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
os.environ["MAPA_FORCE_COLLECTIVES"] = "1"
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 13
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    torch.cuda.set_device(0)
    from mapanything.models import MapAnything
    from mapanything.parallel import ShardPlan, init_distributed
    from mapanything.utils import synthetic
    from tests_helpers import released_config

    init_distributed("nccl", torch.device("cuda", 0))
    model = MapAnything(**released_config()).load_synthetic_weights().to("cuda")
    model.enable_view_sharding(dist.group.WORLD)
    imgs = torch.cat([torch.from_numpy(i) for i in synthetic.synthetic_images(V, 518, 518, 5)], 0).cuda()
    eng = model.engine()
    plan = ShardPlan(V, 1, 0, 37 * 37)
    res = {"views": V}
    with torch.inference_mode():
        for mode in ("eager", "graph"):
            model.hip_graphs = mode == "graph"
            run = (lambda: model._run_engine(eng, imgs, plan, None, None))
            run()
            torch.cuda.synchronize()
            host, wall = [], []
            for _ in range(reps):
                t0 = time.perf_counter()
                run()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                host.append(t1 - t0)
                wall.append(t2 - t0)
            res[mode] = {"host_enqueue_ms": 1e3 * sorted(host)[reps // 2], "wall_ms": 1e3 * sorted(wall)[reps // 2]}
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Repeat the in-thread 3-rank bf16 sharded forward (tests/test_gpu_sharded.py::test_sharded_equals_single[3-3-bf16])
and report, per repetition, which rank / view / output is non-finite and the worst rel-L2 against the single-GPU run.
Usage: python tools/shard_nan_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-anything_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from conftest import rel_l2  # noqa: E402
from mapanything.models import MapAnything  # noqa: E402
from mapanything.parallel import ThreadComm  # noqa: E402
from tests_helpers import released_config  # noqa: E402
from test_gpu_sharded import _run_ranks, _views  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
world, V = 3, 3
views = _views(V, 224, 280, seed=11)
ref_model = MapAnything(**released_config(), precision="bf16").load_synthetic_weights().to("cuda")
ref = ref_model.forward(views)
for rep in range(reps):
    comm = ThreadComm(world)
    model = MapAnything(**released_config(), precision="bf16").to("cuda")
    model._sd = ref_model._sd
    model.enable_view_sharding(comm=comm)
    model.engine()
    outs = _run_ranks(comm, world, lambda rank: model.forward(views))
    bad, worst = [], 0.0
    for r in range(world):
        for v, o in enumerate(outs[r]):
            if o is None:
                continue
            for k in ("pts3d", "conf", "cam_quats", "cam_trans", "metric_scaling_factor"):
                t = o[k].float().cpu()
                if not torch.isfinite(t).all():
                    bad.append((r, v, k, int((~torch.isfinite(t)).sum())))
                else:
                    worst = max(worst, rel_l2(t, ref[v][k].float().cpu()))
    print(f"rep {rep}: non-finite {bad} worst rel-L2 {worst:.2e}", flush=True)

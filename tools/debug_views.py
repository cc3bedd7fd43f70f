"""Debug: V-view job single GPU (graph and eager) vs 8-rank ThreadComm shard; per-view pts3d rel-L2."""
import os
import sys
import threading

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "map-anything_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from mapanything.models import MapAnything  # noqa: E402
from mapanything.parallel import ThreadComm  # noqa: E402
from mapanything.utils import synthetic  # noqa: E402
from tests_helpers import released_config  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


V = int(sys.argv[1]); R = int(sys.argv[2]); world = int(sys.argv[3]); prec = sys.argv[4] if len(sys.argv) > 4 else "bf16"
imgs = synthetic.synthetic_images(V, R, R, 21)
views = [{"img": torch.from_numpy(i), "data_norm_type": ["dinov2"]} for i in imgs]
m = MapAnything(**released_config(), precision=prec).load_synthetic_weights().to("cuda")
g = m.forward(views)
m.hip_graphs = False
e = m.forward(views)
print("graph vs eager", max(rel(g[v]["pts3d"], e[v]["pts3d"]) for v in range(V)), flush=True)
comm = ThreadComm(world)
ms = MapAnything(**released_config(), precision=prec).to("cuda")
ms._sd = m._sd
ms.enable_view_sharding(comm=comm)
ms.engine()
outs = [None] * world
def run(r):
    comm.bind(r)
    outs[r] = ms.forward(views)
th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
[t.start() for t in th]; [t.join() for t in th]
torch.cuda.synchronize()
for r in range(world):
    errs = [(v, round(rel(o["pts3d"], e[v]["pts3d"]), 5)) for v, o in enumerate(outs[r]) if o is not None]
    print("rank", r, errs, flush=True)

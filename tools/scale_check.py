"""Large-N robustness / timing check on one GPU: python tools/scale_check.py <views> [--mem-eff] [--geometric]
Runs MapAnything.infer on <views> synthetic 518x518 views (bf16) and prints time, peak memory and finiteness."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "map-anything_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from mapanything.models import MapAnything  # noqa: E402
from mapanything.utils import synthetic  # noqa: E402
from tests_helpers import released_config  # noqa: E402

V = int(sys.argv[1])
mem_eff = "--mem-eff" in sys.argv
model = MapAnything(**released_config()).load_synthetic_weights().to("cuda").eval()
imgs = synthetic.synthetic_images(V, 518, 518, seed=2)
views = [{"img": torch.from_numpy(i).cuda(), "data_norm_type": ["dinov2"]} for i in imgs]
if "--geometric" in sys.argv:
    Ks = synthetic.synthetic_intrinsics(V, 518, 518, seed=4)
    Ds = synthetic.synthetic_sparse_depth(V, 518, 518, seed=4)
    for v, K, D in zip(views, Ks, Ds):
        v.update(intrinsics=torch.from_numpy(K).cuda(), depth_z=torch.from_numpy(D).cuda())
torch.cuda.synchronize()
torch.cuda.reset_peak_memory_stats()
t0 = time.perf_counter()
out = model.infer(views, memory_efficient_inference=mem_eff)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
finite = all(bool(torch.isfinite(o["pts3d"]).all()) for o in out)
print(f"views={V} mem_eff={mem_eff} seconds={dt:.2f} views/s={V / dt:.1f} "
      f"peak_GB={torch.cuda.max_memory_allocated() / 2**30:.1f} finite={finite}", flush=True)

"""Does the in-thread sharded test's configuration (3 synthetic views at 224x280, bf16 recipe, TF32-equivalent heads)
raise binary16 range faults?  Prints MapAnything.range_fallbacks around one single-GPU forward and one infer."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-anything_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from mapanything.models import MapAnything  # noqa: E402
from mapanything.utils import synthetic  # noqa: E402
from tests_helpers import released_config  # noqa: E402

views = [{"img": torch.from_numpy(i), "data_norm_type": ["dinov2"]} for i in synthetic.synthetic_images(3, 224, 280, 11)]
m = MapAnything(**released_config(), precision="bf16").load_synthetic_weights().to("cuda")
before = MapAnything.range_fallbacks
out = m.forward(views)
torch.cuda.synchronize()
print("range_fallbacks after forward:", MapAnything.range_fallbacks - before,
      "finite:", all(torch.isfinite(o["pts3d"]).all().item() for o in out), flush=True)

"""Input-pipeline throughput: load_images on N synthetic 1280x960 JPEGs -> 518x392 (images/s), host part with
1 worker (the reference's sequential loop) and with the thread pool, plus the GPU normalisation when a GPU is
present.  python tools/bench_inputs.py [N]"""
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "map-anything_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import json  # noqa: E402

import PIL.Image  # noqa: E402
import torch  # noqa: E402

from mapanything.utils.image import load_images, load_resized_images  # noqa: E402
from tests_helpers import synthetic_image  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    with tempfile.TemporaryDirectory() as d:
        for i in range(n):
            PIL.Image.fromarray(synthetic_image(1280, 960, i)).save(os.path.join(d, f"{i:04d}.jpg"), quality=92)
        res = {"images": n, "source": "1280x960 JPEG", "target": "518x392 (fixed_mapping)"}
        for w in (1, None):
            t0 = time.perf_counter()
            load_resized_images(d, num_workers=w)
            dt = time.perf_counter() - t0
            res[f"host_images_per_s_workers_{w or 'auto'}"] = n / dt
        if torch.cuda.is_available():
            load_images(d)  # warm-up (library load, allocator)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            load_images(d)
            torch.cuda.synchronize()
            res["load_images_images_per_s"] = n / (time.perf_counter() - t0)
        print(json.dumps(res))


if __name__ == "__main__":
    main()

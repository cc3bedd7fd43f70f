"""Do the parallel branches of a captured HIP graph run concurrently on this stack?  Two independent small-grid
GEMMs (64 tiles each, long K) captured (a) on one stream, (b) forked onto two streams; replay times compared."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "map-anything_amd"))
import torch  # noqa: E402

from mapanything import _native as nat  # noqa: E402

nat.lib()
dev = torch.device("cuda", 0)
M, N, K = 2048, 1024, 4032  # 128 tiles of 128x128 (K < 4096: no stream-K): half the CUs
A1, A2 = [(torch.randn(M, K, device=dev) * 0.1).bfloat16() for _ in range(2)]
W1, W2 = [(torch.randn(N, K, device=dev) * 0.01).bfloat16() for _ in range(2)]
o1, o2 = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2)]


def one(a, w, o):
    nat.gemm(a, w, M, N, K, out_lp=o)


def serial():
    one(A1, W1, o1)
    one(A2, W2, o2)


side = torch.cuda.Stream(dev)


def forked():
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)
    one(A1, W1, o1)
    with torch.cuda.stream(side):
        one(A2, W2, o2)
    cur.wait_stream(side)


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


res = {}
for name, fn in (("serial", serial), ("forked", forked)):
    res[name + "_eager"] = timed(fn)
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    res[name + "_graph"] = timed(g.replay)
res["single"] = timed(lambda: one(A1, W1, o1))
for k, v in res.items():
    print(f"{k:14s} {v:8.1f} us", flush=True)

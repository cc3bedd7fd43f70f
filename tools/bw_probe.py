"""HBM bandwidth probes next to the path's streaming kernels: torch fill / copy of the regressor resize's output size
(1.1 GB) against mapa_bilinear_ac's split resizes (kbench 'bil').  GPU box: python tools/bw_probe.py"""
import torch


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


n = 8 * 518 * 518 * 256  # bf16 elements of the split 518^2 map
a = torch.empty(n, dtype=torch.bfloat16, device="cuda")
b = torch.empty(n, dtype=torch.bfloat16, device="cuda")
ms = t(lambda: a.fill_(1.0))
print(f"fill  {a.numel()*2/1e9:.2f} GB: {ms*1e3:7.1f} us  {a.numel()*2/ms/1e9:5.2f} TB/s write")
ms = t(lambda: b.copy_(a))
print(f"copy  {a.numel()*2/1e9:.2f} GB: {ms*1e3:7.1f} us  {2*a.numel()*2/ms/1e9:5.2f} TB/s read+write")
x = torch.empty(8 * 296 * 296 * 128, dtype=torch.float32, device="cuda")
ms = t(lambda: x.sum())
print(f"read  {x.numel()*4/1e9:.2f} GB: {ms*1e3:7.1f} us  {x.numel()*4/ms/1e9:5.2f} TB/s read")

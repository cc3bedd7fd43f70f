"""Which hipBLASLt kernels (names encode macro tile / depth / wave layout) torch picks for the path's GEMM shapes."""
import torch

SH = [("enc.qkv", 10960, 3072, 1024), ("enc.proj", 10960, 1024, 1024), ("enc.fc1", 10960, 4096, 1024),
      ("enc.fc2", 10960, 1024, 4096), ("aat.qkv", 10953, 2304, 768), ("aat.proj", 10953, 768, 768),
      ("aat.fc1", 10953, 3072, 768), ("aat.fc2", 10953, 768, 3072)]
for name, M, N, K in SH:
    A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    for _ in range(5):
        torch.nn.functional.linear(A, W, b)
    torch.cuda.synchronize()
print("ok")

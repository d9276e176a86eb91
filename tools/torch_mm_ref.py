"""Reference point for the chunk GEMM (development tool): torch.bmm fp32
(hipBLASLt / rocBLAS inside torch) on the shape of tools/gemm_probe.py,
8 x 5000^3 f32 products, TF32 off."""
import torch

n, T = 5000, 8
A = torch.rand(T, n, n, device="cuda") - 0.5
B = torch.rand(T, n, n, device="cuda") - 0.5
torch.backends.cuda.matmul.allow_tf32 = False
C = torch.bmm(A, B)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    C = torch.bmm(A, B)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
print(f"torch.bmm fp32: {ms:.2f} ms {2 * T * n ** 3 / ms / 1e9:.1f} TF")

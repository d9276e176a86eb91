"""Vendor reference point for the chained GEMM (development tool):
torch.matmul (hipBLASLt / rocBLAS inside PyTorch) on BASELINE config 5's
operands as ONE unchunked 40000^2 x 40000^2 product, f32 (TF32 off; gfx950
has no xf32 anyway) and bf16, uniform [-1, 1) data, best of 3 after a
warm-up.  The chained kernel does the same flops on 5000^2 chunk slots
(64 output chunks x 8 segments); this times the library on a plain
contiguous problem of the same size."""
import torch

n = 40000
torch.backends.cuda.matmul.allow_tf32 = False
for dt in (torch.float32, torch.bfloat16):
    A = (torch.rand(n, n, device="cuda", dtype=torch.float32) * 2 - 1).to(dt)
    B = (torch.rand(n, n, device="cuda", dtype=torch.float32) * 2 - 1).to(dt)
    C = torch.matmul(A, B)
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        C = torch.matmul(A, B)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    print(f"torch.matmul {str(dt).split('.')[-1]} {n}^3: {best:.2f} ms {2 * n ** 3 / best / 1e9:.1f} TF", flush=True)
    del A, B, C
    torch.cuda.empty_cache()

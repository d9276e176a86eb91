"""GEMM probe (development tool): cubed_gemm_chunks on 8 f32 5000^3 chunk
products, TFLOP/s and max error vs an f64 product.  (Variants were selected
through a temporary CUBED_GEMM_VARIANT switch while tuning; see gemm.hip.)"""
import os
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import numpy as np
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from cubed_amd import _native as nat

    n, T = 5000, 8
    A = torch.rand(T, n, n, device="cuda") - 0.5
    B = torch.rand(T, n, n, device="cuda") - 0.5
    C = torch.empty(T, n, n, device="cuda")
    rows = np.zeros(T, dtype=nat.GEMM_DTYPE)
    for t in range(T):
        rows[t] = (A[t].data_ptr(), B[t].data_ptr(), C[t].data_ptr(), n, n, n, n, n, n, 0)
    tab = torch.from_numpy(rows.view(np.uint8).copy()).cuda()
    L = nat.lib()
    st = torch.cuda.current_stream().cuda_stream
    if os.environ.get("CUBED_GEMM_VARIANT") == "blas":
        from cubed_amd.lowering import GemmLaunch

        GL = GemmLaunch(rows, 9, n, n, torch.device("cuda"))
        assert GL.blas
        run = lambda: GL.run(st)  # noqa: E731
    else:
        run = lambda: nat.check(L.cubed_gemm_chunks(tab.data_ptr(), T, 9, n, n, st), "gemm")  # noqa: E731
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    ref = (A[0].double() @ B[0].double()).float()
    err = (C[0] - ref).abs().max().item()
    print(f"variant {os.environ.get('CUBED_GEMM_VARIANT', '0')}: {ms:.2f} ms, "
          f"{2 * T * n ** 3 / ms / 1e9:.1f} TF, max err {err:.2e}", flush=True)
else:
    for v in sys.argv[1:] or ["0"]:
        env = dict(os.environ, CUBED_GEMM_VARIANT=v)  # "blas" = rocBLAS path, else the native kernel
        subprocess.run([sys.executable, __file__, "--child"], env=env, check=True, timeout=300)

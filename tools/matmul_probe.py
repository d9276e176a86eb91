"""Matmul probe (development tool): BASELINE config 5 through the drop-in API
-- xp.matmul of two (n, n) arrays in (c, c) chunks, f32 and/or bf16 -- timed
per plan execution and per GEMM launch (HIP events), with a sampled check of
the first output rows against an f64 product of the same (rounded) inputs.

    python tools/matmul_probe.py [--n 40000] [--c 5000] [--dtypes f32,bf16] [--reps 2]
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TF = {"f32": 157.3, "bf16": 2500.0}  # MI355X dense MFMA peaks (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=40000)
    ap.add_argument("--c", type=int, default=5000)
    ap.add_argument("--dtypes", default="f32,bf16")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--check-rows", type=int, default=16)
    ap.add_argument("--unfused", action="store_true", help="reference plan: per-chunk products + k-sum")
    args = ap.parse_args()

    import numpy as np
    import torch

    import cubed_amd as cubed
    import cubed_amd.array_api as xp
    import cubed_amd.random as crandom
    from cubed_amd import ir
    from cubed_amd.core.plan import arrays_to_plan
    from cubed_amd.runtime.executors.gpu import GpuDagExecutor, LaunchTimer
    from cubed_amd.storage import DeviceArray

    for dt in args.dtypes.split(","):
        ex = GpuDagExecutor("cuda:0")
        ex.fuse_gemm_sums = not args.unfused
        spec = cubed.Spec(allowed_mem="288GB", executor=ex)
        random.seed(4000)
        xdt = xp.bfloat16 if dt == "bf16" else xp.float32
        A = xp.astype(crandom.random((args.n, args.n), chunks=(args.c, args.c), spec=spec), xdt)
        B = xp.astype(crandom.random((args.n, args.n), chunks=(args.c, args.c), spec=spec), xdt)
        arrays_to_plan(A, B).execute(executor=ex, array_names=[A.name, B.name])
        torch.cuda.synchronize()
        m = xp.matmul(A, B)
        plan = arrays_to_plan(m)
        keep = {id(A.zarray), id(B.zarray)}

        def step():
            for _, d in plan._finalize_dag().nodes(data=True):
                t = d.get("target")
                if isinstance(t, DeviceArray) and id(t) not in keep:
                    t.written = False
            plan.execute(executor=ex, resume=True, array_names=[m.name])

        step()
        torch.cuda.synchronize()
        ex.timing = LaunchTimer()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            step()
        torch.cuda.synchronize()
        dt_s = (time.perf_counter() - t0) / args.reps
        summ = ex.timing.summary()
        ex.timing = None
        flop = 2.0 * args.n ** 3
        gemm = {f"{k[0]}#{k[1]}": v[1] for k, v in summ.items() if k[2] == "GemmLaunch"}
        gms = sum(gemm.values())
        out = dict(dtype=dt, n=args.n, chunk=args.c, plan_ms=round(dt_s * 1e3, 2),
                   plan_tflops=round(flop / dt_s / 1e12, 1), gemm_ms=round(gms, 2),
                   gemm_tflops=round(flop / (gms * 1e-3) / 1e12, 1) if gms else None,
                   launches={f"{k[0]}#{k[1]}:{k[2]}": round(v[1], 3) for k, v in summ.items()})
        if gms:
            out["frac_of_peak"] = round(out["gemm_tflops"] / PEAK_TF[dt], 4)
        # sampled check: first rows of output chunk (0, 0) against f64
        r = args.check_rows
        Ad, Bd, Md = A.zarray, B.zarray, m.zarray
        conv = (lambda v: ir.bf16_to_numpy(v)) if dt == "bf16" else (lambda v: v)
        nk = args.n // args.c
        arow = np.concatenate([conv(Ad.read_chunk((0, k)))[:r] for k in range(nk)], axis=1).astype(np.float64)
        bcol = np.concatenate([conv(Bd.read_chunk((k, 0))) for k in range(nk)], axis=0).astype(np.float64)
        got = conv(Md.read_chunk((0, 0)))[:r].astype(np.float64)
        exp = arow @ bcol
        scale = np.abs(arow) @ np.abs(bcol)
        rel = np.abs(got - exp) / scale
        out["check"] = dict(rows=r, max_rel_err=float(rel.max()),
                            bound_8sqrtK_u=8 * np.sqrt(args.n) * 2.0 ** -24 + (2.0 ** -8 if dt == "bf16" else 0))
        print(json.dumps(out), flush=True)
        del A, B, m, plan, ex
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Development probe (not part of the library): what makes config 3's rechunk
copy (2500 boxes of 1000 x 1000 f32, source rows at a 200000-B stride,
destination contiguous: k_copy_flat) run 3.35 or 3.85 ms.  Round 3/4 saw the
same box tables take either time depending on which buffers they ran on
(profiles/r03_copy_placement.log), with equal UTCL1 counters
(r04_copy_tlb_pmc.log).  Here the source and target live in ONE arena at
chosen offsets, so every placement is reproducible:

  * sweep the target's offset relative to the source (delta),
  * swap the order (target below source),
  * fresh torch allocations (the executor's current placement) as control.

Run on the GPU box:  python tools/copy_arena_probe.py [reps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cubed_amd.lowering import Box, CopyLaunch  # noqa: E402

N, C = 50000, 1000
SLOT = C * N * 4           # one (1000, 50000) f32 row chunk = one (50000, 1000) column chunk
NB = N // C
TOTAL = NB * SLOT          # 1e10 B


def boxes(src, dst):
    out = []
    for i in range(NB):          # source row chunk
        for j in range(NB):      # target column chunk
            out.append(Box(src + i * SLOT + j * C * 4, dst + j * SLOT + i * C * C * 4,
                           [C, C], [N, 1], [C, 1]))
    out.sort(key=lambda b: b.src)
    return out


def time_copy(src, dst, reps):
    L = CopyLaunch(boxes(src, dst), 4, torch.device("cuda"))
    s = torch.cuda.current_stream()
    for _ in range(2):
        L.run(s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        L.run(s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    pad = 1 << 30
    arena = torch.empty(2 * TOTAL + 2 * pad, dtype=torch.uint8, device="cuda")
    base = (arena.data_ptr() + (1 << 21) - 1) // (1 << 21) * (1 << 21)  # 2 MiB aligned
    arena.view(torch.int32)[: (2 * TOTAL) // 4].copy_(
        torch.arange((2 * TOTAL) // 4, dtype=torch.int32, device="cuda") * 2654435761)
    torch.cuda.synchronize()
    print(f"arena base {base:#x} (2 MiB aligned)", flush=True)
    ten = (TOTAL + (1 << 21) - 1) // (1 << 21) * (1 << 21)
    for delta in (0, 256, 4096, 65536, 1 << 20, 1 << 21, (1 << 21) + 4096, 3 << 20, 1 << 24,
                  (1 << 24) + (1 << 20), 1 << 28, 1 << 29, 3 << 28):
        ms = time_copy(base, base + ten + delta, reps)
        print(f"src=base       dst=base+{ten:#x}+{delta:#x}: {ms:.4f} ms  ({2 * TOTAL / ms / 1e6:.0f} GB/s moved)",
              flush=True)
    for delta in (0, 4096, 1 << 21, 1 << 28):
        ms = time_copy(base + ten + delta, base, reps)
        print(f"dst=base       src=base+{ten:#x}+{delta:#x}: {ms:.4f} ms", flush=True)
    for so in (4096, 1 << 20, 1 << 21, 1 << 28):
        ms = time_copy(base + so, base + so + ten + (1 << 21), reps)
        print(f"src=base+{so:#x} dst=src+{ten:#x}+0x200000: {ms:.4f} ms", flush=True)
    # physical placement: several arenas held at once occupy different HBM
    # pages; the same copy in each (and across them)
    arenas = [arena]
    for _ in range(int(os.environ.get("ARENAS", "4"))):
        a = torch.empty(2 * TOTAL + 2 * pad, dtype=torch.uint8, device="cuda")
        a.view(torch.int32)[: (2 * TOTAL) // 4].fill_(7)
        arenas.append(a)
    torch.cuda.synchronize()
    bases = [(a.data_ptr() + (1 << 21) - 1) // (1 << 21) * (1 << 21) for a in arenas]
    for rep in range(2):
        for k, b in enumerate(bases):
            ms = time_copy(b, b + ten, reps)
            print(f"arena {k} ({b:#x}): {ms:.4f} ms", flush=True)
    for k in range(1, len(bases)):
        ms = time_copy(bases[0], bases[k] + ten, reps)
        print(f"src arena 0, dst arena {k}: {ms:.4f} ms", flush=True)
    # box references in the same process: hipMemcpy D2D of 10 GB, a read-only sum
    x = arenas[0][:TOTAL]
    y = arenas[1][:TOTAL]
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    y.copy_(x)
    e0.record(s)
    for _ in range(reps):
        y.copy_(x)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"reference: torch D2D copy of 1e10 B: {ms:.4f} ms ({2 * TOTAL / ms / 1e6:.0f} GB/s moved)", flush=True)
    del arenas, arena, x, y
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    for k in range(4):  # fresh torch allocations, as the executor makes them
        x = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
        y = torch.empty(TOTAL, dtype=torch.uint8, device="cuda")
        x.view(torch.int32).copy_(torch.arange(TOTAL // 4, dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        ms = time_copy(x.data_ptr(), y.data_ptr(), reps)
        print(f"fresh pair {k}: src {x.data_ptr():#x} dst {y.data_ptr():#x} (dst-src {y.data_ptr() - x.data_ptr():#x}): "
              f"{ms:.4f} ms", flush=True)
        ms2 = time_copy(y.data_ptr(), x.data_ptr(), reps)
        print(f"    swapped: {ms2:.4f} ms", flush=True)
        del x, y
        time.sleep(0.2)


if __name__ == "__main__":
    main()

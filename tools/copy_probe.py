"""Probe of cubed_copy_boxes rates on MI355X (development tool): a plain
contiguous copy vs the rechunk pattern of BASELINE config 3, same bytes."""
import ctypes
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cubed_amd import _native as nat
from cubed_amd.lowering import Box, CopyLaunch


def run(name, boxes, isz, nbytes, reps=5):
    L = CopyLaunch(boxes, isz, torch.device("cuda:0"))
    st = torch.cuda.current_stream().cuda_stream
    L.run(st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.run(st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name}: {ms:.3f} ms, {2 * nbytes / ms / 1e6:.0f} GB/s (read+write), path {L.path} lane {L.lane} "
          f"work {L.work} row_bytes {L.row_bytes} nboxes {L.nboxes}", flush=True)


N = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
C = 1000
src = torch.empty(N * N * 4, dtype=torch.uint8, device="cuda")
dst = torch.empty(N * N * 4, dtype=torch.uint8, device="cuda")
sb, db = src.data_ptr(), dst.data_ptr()
nbytes = N * N * 4
# (a) contiguous: rows of 4096 B, one box per 64 MiB
rows = nbytes // 4096
per = 16384
boxes = [Box(sb + i * 4096, db + i * 4096, [min(per, rows - i), 4096], [4096, 1], [4096, 1])
         for i in range(0, rows, per)]
run("contiguous 4KiB rows", boxes, 1, nbytes)
# (b) rechunk rows (1000, N) -> cols (N, 1000), f32 elements
boxes = []
for i in range(N // C):          # source chunk i: rows [iC, iC+C), slot i
    for j in range(N // C):      # target chunk j: cols [jC, jC+C), slot j
        s = sb + (i * C * N + j * C) * 4
        d = db + (j * N * C + i * C * C) * 4
        boxes.append(Box(s, d, [C, C], [N, 1], [C, 1]))
run("rechunk boxes", boxes, 4, nbytes)
# (c) same box structure as (b), sequential addresses on both sides
boxes = []
for i in range(N // C):
    for j in range(N // C):
        o = (i * (N // C) + j) * C * C * 4
        boxes.append(Box(sb + o, db + o, [C, C], [C, 1], [C, 1]))
run("rechunk-shaped boxes, sequential", boxes, 4, nbytes)
# (d) rechunk, boxes ordered source-row-major (a block's neighbours read the same rows)
boxes = []
for i in range(N // C):
    for r0 in range(0, C, 8):
        for j in range(N // C):
            s = sb + ((i * C + r0) * N + j * C) * 4
            d = db + (j * N * C + (i * C + r0) * C) * 4
            boxes.append(Box(s, d, [8, C], [N, 1], [C, 1]))
run("rechunk 8-row boxes, source order", boxes, 4, nbytes)

"""Helpers to run a function on N ranks of a local process group (gloo by
default), for the multi-GPU tests: ``run_ranks(fn, world, *args)`` spawns
``world`` processes, each calling ``fn(rank, world, *args)`` after
``init_process_group``, and raises if any rank fails or hangs."""

import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, backend, fn, args, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group(backend, rank=rank, world_size=world)
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
    except BaseException:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "error", traceback.format_exc()))
    finally:
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass


def run_ranks(fn, world, *args, backend="gloo", timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, backend, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            results[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]


def host_copy(cl):
    """Run a CopyLaunch's boxes on the HOST (CPU-tensor tests of launches
    whose copies the library runs on the GPU): element by element, with the
    canonical boxes' strides."""
    import ctypes
    import itertools

    if cl.nboxes == 0:
        return
    isz = cl.itemsize
    for b in cl.boxes:
        for idx in itertools.product(*[range(e) for e in b.extent]):
            so = sum(i * s for i, s in zip(idx, b.sstride)) * isz
            do = sum(i * s for i, s in zip(idx, b.dstride)) * isz
            ctypes.memmove(b.dst + do, b.src + so, isz)

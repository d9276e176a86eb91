"""Multi-GPU exchange plans (cubed_amd/runtime/exchange.py) and the
collective layer (cubed_amd/runtime/comm.py), on CPU.

The plans are pure chunk geometry, so they are checked exhaustively here:
every target element is written exactly once, and what rank s packs for
rank d is exactly what d unpacks from s.  The data path is then driven over
a real gloo process group (world 2 and 3) with numpy standing in for the
pack/unpack box copies the GPU executor runs as HIP kernels -- the bytes
that cross ranks, their order and the split sizes are the product's own.
"""

import itertools
import math

import numpy as np
import pytest

from cubed_amd.runtime.exchange import (
    owner_of,
    plan_fetch,
    plan_rechunk,
    rechunk_pieces,
    round_up,
)
from cubed_amd.storage import ChunkGrid
from distutil import run_ranks

CASES = [
    ((12, 10), (5, 10), (12, 3)),        # row chunks -> column chunks (config 3 shape)
    ((12, 10), (4, 4), (3, 7)),          # misaligned both ways, edge chunks
    ((7, 5, 6), (2, 5, 6), (7, 2, 3)),   # 3-d
    ((9,), (2,), (4,)),
    ((10, 10), (10, 10), (1, 10)),       # one source chunk
]


def grids(case, dtype=np.float32):
    shape, a, b = case
    return ChunkGrid(shape, dtype, a), ChunkGrid(shape, dtype, b)


@pytest.mark.parametrize("case", CASES)
def test_pieces_tile_every_target_once(case):
    src, dst = grids(case)
    cover = np.zeros(src.shape, dtype=np.int32)
    for p in rechunk_pieces(src, dst):
        start = [s + o for s, o in zip(dst.chunk_start(p.dst), p.dst_start)]
        sstart = [s + o for s, o in zip(src.chunk_start(p.src), p.src_start)]
        assert start == sstart  # same global position on both sides
        cover[tuple(slice(s, s + e) for s, e in zip(start, p.extent))] += 1
        for d in range(src.ndim):  # inside both chunks
            assert p.src_start[d] + p.extent[d] <= src.chunk_extent(p.src)[d]
            assert p.dst_start[d] + p.extent[d] <= dst.chunk_extent(p.dst)[d]
    assert (cover == 1).all()


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rechunk_plans_agree_between_ranks(case, world):
    src, dst = grids(case)
    plans = [plan_rechunk(src, dst, r, world, 4) for r in range(world)]
    total = sum(p.size for p in rechunk_pieces(src, dst))
    moved = 0
    for s in range(world):
        for d in range(world):
            sent = plans[s].send[d]
            got = plans[d].recv[s]
            assert [p for p, _ in sent] == [p for p, _ in got]
            assert plans[s].send_splits[d] == plans[d].recv_splits[s]
            assert plans[s].send_splits[d] == sum(round_up(p.size * 4) for p, _ in sent)
            for p, _ in sent:
                assert owner_of(src, p.src, world) == s and owner_of(dst, p.dst, world) == d
            moved += sum(p.size for p, _ in sent)
        moved += sum(p.size for p in plans[s].local)
    assert moved == total
    if world == 1:
        assert not plans[0].exchanges


def test_replicated_source_is_all_local():
    src, dst = grids(CASES[1])
    for r in range(3):
        plan = plan_rechunk(src, dst, r, 3, 4, src_world=1)
        assert not plan.exchanges
        assert all(owner_of(dst, p.dst, 3) == r for p in plan.local)


def test_fetch_plan_consistency():
    g = ChunkGrid((8, 8), np.float64, (2, 2))
    world = 3
    # every rank reads a few chunks (some its own)
    needs = {r: {("x", c, None) for c in itertools.product(range(4), range(4))
                 if (c[0] + c[1] + r) % 3 == 0} for r in range(world)}
    owner = lambda ref: g.chunk_offset(ref[1]) % world  # noqa: E731
    nbytes = lambda ref: math.prod(g.chunk_extent(ref[1])) * 8  # noqa: E731
    plans = [plan_fetch(needs, owner, nbytes, r, world) for r in range(world)]
    for s in range(world):
        for d in range(world):
            assert [x[0] for x in plans[s].send[d]] == [x[0] for x in plans[d].recv[s]]
            assert plans[s].send_splits[d] == plans[d].recv_splits[s]
        for ref, _, _ in itertools.chain(*plans[s].recv):
            assert owner(ref) != s and ref in needs[s]
        assert {ref for ref in needs[s] if owner(ref) != s} == \
            {ref for ref, _, _ in itertools.chain(*plans[s].recv)}


# ---------------------------------------------------------------- gloo data path


def _rechunk_rank(rank, world, case):
    import torch

    from cubed_amd.runtime.comm import Comm

    comm = Comm()
    src, dst = grids(case)
    full = np.arange(math.prod(src.shape), dtype=np.float32).reshape(src.shape)

    def chunk(grid, c):
        return tuple(slice(s, s + e) for s, e in zip(grid.chunk_start(c), grid.chunk_extent(c)))

    mine = {c: full[chunk(src, c)].copy() for c in itertools.product(*map(range, src.numblocks))
            if owner_of(src, c, world) == rank}
    out = {c: np.full(dst.chunk_extent(c), -1, np.float32)
           for c in itertools.product(*map(range, dst.numblocks)) if owner_of(dst, c, world) == rank}
    plan = plan_rechunk(src, dst, rank, world, 4)
    send = np.zeros(max(plan.send_bytes, 16), np.uint8)
    for lst in plan.send:
        for p, off in lst:
            box = mine[p.src][tuple(slice(a, a + e) for a, e in zip(p.src_start, p.extent))]
            send[off:off + box.nbytes] = np.ascontiguousarray(box).view(np.uint8).reshape(-1)
    recv = torch.zeros(max(plan.recv_bytes, 16), dtype=torch.uint8)
    comm.all_to_all(recv, torch.from_numpy(send), plan.recv_splits, plan.send_splits)
    rb = recv.numpy()
    for p in plan.local:
        out[p.dst][tuple(slice(a, a + e) for a, e in zip(p.dst_start, p.extent))] = \
            mine[p.src][tuple(slice(a, a + e) for a, e in zip(p.src_start, p.extent))]
    for lst in plan.recv:
        for p, off in lst:
            n = p.size * 4
            out[p.dst][tuple(slice(a, a + e) for a, e in zip(p.dst_start, p.extent))] = \
                rb[off:off + n].view(np.float32).reshape(p.extent)
    for c, v in out.items():
        assert np.array_equal(v, full[chunk(dst, c)]), (rank, c)
    return len(out)


@pytest.mark.parametrize("world", [2, 3])
def test_rechunk_exchange_over_gloo(world):
    for case in CASES[:3]:
        counts = run_ranks(_rechunk_rank, world, case)
        src, dst = grids(case)
        assert sum(counts) == math.prod(dst.numblocks)


def _reduce_rank(rank, world):
    import torch

    from cubed_amd.runtime.comm import Comm

    comm = Comm()
    n = 10
    tot = torch.full((n,), float(rank + 1), dtype=torch.float64)
    cnt = torch.full((n,), rank + 2, dtype=torch.int64)
    comm.reduce_sum(tot, 0)
    comm.all_reduce_sum(cnt)
    parts = torch.zeros(world * n, dtype=torch.float64)
    comm.all_gather(parts, torch.arange(n, dtype=torch.float64) * (rank + 1))
    b = torch.tensor([7.0 if rank == 1 else 0.0], dtype=torch.float64)
    comm.broadcast(b, 1)
    return tot.tolist(), cnt.tolist(), parts.view(world, n).tolist(), b.item()


def test_partials_collectives_over_gloo():
    world = 3
    res = run_ranks(_reduce_rank, world)
    tot0, cnt0, parts0, b0 = res[0]
    assert tot0 == [6.0] * 10                    # 1 + 2 + 3 on the root
    assert all(r[1] == [2 + 3 + 4] * 10 for r in res)
    assert parts0 == [[i * (r + 1) for i in range(10)] for r in range(world)]
    assert all(r[3] == 7.0 for r in res)

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
    box_contiguous,
    box_offset,
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
            # both ends post the pair's transfers in the same order and sizes
            assert [(x.piece, x.index, x.nbytes) for x in sent] == [(x.piece, x.index, x.nbytes) for x in got]
            assert [x.index for x in sent] == sorted(x.index for x in sent)
            for x in sent:
                p = x.piece
                assert owner_of(src, p.src, world) == s and owner_of(dst, p.dst, world) == d
                assert x.nbytes == p.size * 4
                assert x.direct == box_contiguous(src.chunk_extent(p.src), p.src_start, p.extent)
            for x in got:
                p = x.piece
                assert x.direct == box_contiguous(dst.chunk_extent(p.dst), p.dst_start, p.extent)
            moved += sum(x.piece.size for x in sent)
        moved += sum(p.size for p in plans[s].local)
        # packed / staged pieces get disjoint 256-B aligned buffer ranges
        for lst, size in ((plans[s].send, plans[s].pack_bytes), (plans[s].recv, plans[s].stage_bytes)):
            spans = sorted((x.offset, x.offset + x.nbytes) for l in lst for x in l if not x.direct)
            assert all(a % 256 == 0 for a, _ in spans)
            assert all(b1 <= a2 for (_, b1), (a2, _) in zip(spans, spans[1:]))
            assert all(b <= size for _, b in spans)
    assert moved == total
    if world == 1:
        assert not plans[0].exchanges


def test_row_bands_of_column_chunks_land_in_place():
    """Config 3's shape: every piece (a row band of a source row chunk x the
    target's columns) is one contiguous run of its target column chunk, so
    nothing is staged (no unpack pass); the sources are strided (packed)."""
    src, dst = ChunkGrid((40, 40), np.float32, (5, 40)), ChunkGrid((40, 40), np.float32, (40, 5))
    for world in (2, 8):
        for r in range(world):
            plan = plan_rechunk(src, dst, r, world, 4)
            assert plan.stage_bytes == 0 and all(x.direct for l in plan.recv for x in l)
            assert all(not x.direct for l in plan.send for x in l)
            assert plan.pack_bytes == sum(round_up(x.nbytes) for l in plan.send for x in l)


def test_box_contiguity():
    assert box_contiguous((10, 8), (3, 0), (4, 8))       # whole rows
    assert box_contiguous((10, 8), (3, 2), (1, 5))       # part of one row
    assert not box_contiguous((10, 8), (3, 2), (2, 5))   # parts of two rows
    assert box_contiguous((4, 6, 8), (1, 0, 0), (2, 6, 8))
    assert box_contiguous((4, 6, 8), (1, 2, 0), (1, 3, 8))
    assert not box_contiguous((4, 6, 8), (1, 2, 0), (2, 3, 8))
    assert box_offset((4, 6, 8), (1, 2, 3)) == 1 * 48 + 2 * 8 + 3


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


def _rechunk_rank(rank, world, case, nslices):
    """RechunkLaunch's data path with numpy box copies in place of the pack /
    unpack / local HIP copies: chunk slots are byte tensors, direct transfers
    are views of them (the bytes land in the target slot), the rest go
    through the pack and staging buffers; slices are started in order and
    waited for at the end, as RechunkLaunch.run does."""
    import torch

    from cubed_amd.runtime.comm import Comm

    comm = Comm()
    src, dst = grids(case)
    full = np.arange(math.prod(src.shape), dtype=np.float32).reshape(src.shape)

    def chunk(grid, c):
        return tuple(slice(s, s + e) for s, e in zip(grid.chunk_start(c), grid.chunk_extent(c)))

    def box(p_start, extent):
        return tuple(slice(a, a + e) for a, e in zip(p_start, extent))

    mine = {c: torch.from_numpy(full[chunk(src, c)].copy().reshape(-1).view(np.uint8))
            for c in itertools.product(*map(range, src.numblocks)) if owner_of(src, c, world) == rank}
    out = {c: torch.full((math.prod(dst.chunk_extent(c)) * 4,), 255, dtype=torch.uint8)
           for c in itertools.product(*map(range, dst.numblocks)) if owner_of(dst, c, world) == rank}

    def as_array(buf, grid, c):
        return buf.numpy().view(np.float32).reshape(grid.chunk_extent(c))

    plan = plan_rechunk(src, dst, rank, world, 4)
    pack = torch.zeros(max(plan.pack_bytes, 16), dtype=torch.uint8)
    stage = torch.zeros(max(plan.stage_bytes, 16), dtype=torch.uint8)
    pending = []
    for lo, hi in plan.slice_bounds(nslices):
        sends, recvs = [], []
        for peer, lst in enumerate(plan.send):
            for x in (x for x in lst if lo <= x.index < hi):
                p = x.piece
                if x.direct:
                    o = box_offset(src.chunk_extent(p.src), p.src_start) * 4
                    sends.append((mine[p.src][o:o + x.nbytes], peer))
                else:
                    vals = as_array(mine[p.src], src, p.src)[box(p.src_start, p.extent)]
                    pack[x.offset:x.offset + x.nbytes] = torch.from_numpy(
                        np.ascontiguousarray(vals).reshape(-1).view(np.uint8))
                    sends.append((pack[x.offset:x.offset + x.nbytes], peer))
        for peer, lst in enumerate(plan.recv):
            for x in (x for x in lst if lo <= x.index < hi):
                p = x.piece
                if x.direct:
                    o = box_offset(dst.chunk_extent(p.dst), p.dst_start) * 4
                    recvs.append((out[p.dst][o:o + x.nbytes], peer))
                else:
                    recvs.append((stage[x.offset:x.offset + x.nbytes], peer))
        pending.append(comm.exchange(sends, recvs))
    for p in plan.local:
        as_array(out[p.dst], dst, p.dst)[box(p.dst_start, p.extent)] = \
            as_array(mine[p.src], src, p.src)[box(p.src_start, p.extent)]
    for h in pending:
        h.wait()
    for lst in plan.recv:
        for x in (x for x in lst if not x.direct):
            p = x.piece
            as_array(out[p.dst], dst, p.dst)[box(p.dst_start, p.extent)] = \
                stage[x.offset:x.offset + x.nbytes].numpy().view(np.float32).reshape(p.extent)
    for c, v in out.items():
        assert np.array_equal(as_array(v, dst, c), full[chunk(dst, c)]), (rank, c)
    return len(out)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("nslices", [1, 3])
def test_rechunk_exchange_over_gloo(world, nslices):
    for case in CASES[:3]:
        counts = run_ranks(_rechunk_rank, world, case, nslices)
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


def _agree_rank(rank, world):
    import torch.distributed as dist

    from cubed_amd.runtime.comm import Comm

    comm = Comm()
    assert comm.ctrl is None  # a gloo world needs no separate control group
    # the control-plane path (a host-side gloo group beside a device group)
    comm.ctrl = dist.new_group(backend="gloo")
    comm.staged = False
    return comm.all_ok(True), comm.all_ok(rank != 1), comm.all_ok(True)


def test_agreement_over_the_control_group():
    """Comm.all_ok: plan-time agreements (MIN over ranks) run on the host-side
    gloo group when the data group is RCCL, so they never wait on the GPU
    stream; every rank gets the same answers, in call order."""
    res = run_ranks(_agree_rank, 3)
    assert res == [(True, False, True)] * 3


def _ctrl_once_rank(rank, world):
    import torch.distributed as dist

    import cubed_amd.runtime.comm as C

    made = []
    real = dist.new_group

    def counting(*a, **k):
        made.append(1)
        return real(*a, **k)

    dist.new_group = counting
    try:
        g1 = C.control_group(dist)
        g2 = C.control_group(dist)  # a second executor's Comm: no new group
    finally:
        dist.new_group = real
    return len(made), g1 is g2, g1 is not None


def test_control_group_is_made_once_per_process():
    """one gloo control group per process and world group (every
    default_executor() used to open another one)."""
    assert run_ranks(_ctrl_once_rank, 2) == [(1, True, True)] * 2


def _ctrl_fail_rank(rank, world):
    import torch.distributed as dist

    import cubed_amd.runtime.comm as C

    real = dist.new_group

    def flaky(*a, **k):
        g = real(*a, **k)  # collective: every rank takes part
        if rank == 1:
            raise RuntimeError("no gloo here")
        return g

    dist.new_group = flaky
    try:
        C._CTRL.clear()
        return C.control_group(dist) is None
    finally:
        dist.new_group = real


def test_control_group_failure_is_agreed():
    """If the gloo group cannot be made on one rank, EVERY rank falls back to
    the device group (otherwise all_ok would run on different groups)."""
    assert run_ranks(_ctrl_fail_rank, 2) == [True, True]


# ------------------------------------------------ reduce-scatter combine


def _scatter_rank(rank, world, G, mko):
    """ScatterCombine over gloo with CPU tensors: each rank's SoA partials
    ([count][total] x G groups x mko) hold (rank + 1) * (g + 1) in every
    total; the finish is patched to capture the buffer it would run on."""
    import types

    import torch

    import cubed_amd.runtime.executors.dist as D
    from cubed_amd.lowering import Layout, TaskRow
    from cubed_amd.runtime.comm import Comm

    comm = Comm()
    ctx = types.SimpleNamespace(world=world, rank=rank, device=torch.device("cpu"), comm=comm)
    owner = [g % world for g in range(G)]
    rows = Layout(order=[0], groups=[[0]], ndim=1, nred=0, mode=0, max_kept=mko, max_red=1,
                  rows=[TaskRow([mko], [0], [[1]], [1000 + g], [[1]], 0, 0, 0) for g in range(G)])
    counts = [50 + g for g in range(G)]
    assert D.ScatterCombine.plan(["count", "sum"], True, [True, False]) == (1, 2)
    from distutil import host_copy

    soa = torch.zeros(2 * G * mko, dtype=torch.float64)
    soa.view(2, G, mko)[1] = torch.tensor([(rank + 1.0) * (g + 1) for g in range(G)])[:, None]
    sc = D.ScatterCombine(ctx, None, rows, owner, 2, mko, 1, 2, False, {0: counts}, discard=7, src=soa.data_ptr())
    sc.permute.run = lambda stream: host_copy(sc.permute)  # the owner-major box copy, on the host
    seen = []
    real = D.fused_finish
    D.fused_finish = lambda F, table, nt, mk, part, st: seen.append((nt, mk, part.clone()))
    try:
        sc.run(0)
    finally:
        D.fused_finish = real
    out = {"mine": sc.mine, "L": sc.L, "finished": len(seen)}
    if seen:
        nt, mk, part = seen[0]
        fin = part.view(torch.int64).view(2, sc.L, mko)
        out["counts"] = fin[0, :, 0].tolist()
        out["totals"] = fin[1].view(torch.float64)[:, 0].tolist()
        out["obases"] = [int(x) for x in np.frombuffer(sc.table.numpy().tobytes(), dtype=__import__(
            "cubed_amd._native", fromlist=["TASK_DTYPE"]).TASK_DTYPE)["out_base"][:, 0]]
    return out


@pytest.mark.parametrize("world,G", [(2, 5), (3, 7), (4, 2)])
def test_scatter_combine_over_gloo(world, G):
    """Each rank ends with the SUM over ranks of exactly its own blocks
    (owner-major slots, padding to the busiest rank), the host counts of its
    blocks, a finish table of its blocks (+ padding rows to the discard
    buffer) -- and ranks owning no block run no finish."""
    mko = 3
    res = run_ranks(_scatter_rank, world, G, mko)
    tri = world * (world + 1) / 2
    L = -(-G // world)
    for r, out in enumerate(res):
        mine = [g for g in range(G) if g % world == r]
        assert out["mine"] == mine and out["L"] == max(1, L)
        assert out["finished"] == (1 if mine else 0)
        if mine:
            pad = out["L"] - len(mine)
            assert out["totals"][:len(mine)] == [tri * (g + 1) for g in mine]
            assert out["totals"][len(mine):] == [0.0] * pad
            assert out["counts"] == [50 + g for g in mine] + [1] * pad
            assert out["obases"] == [1000 + g for g in mine] + [7] * pad

"""Lowering of the multi-GPU executor, checked on CPU for every rank of a
world (DryExecutor with a FakeComm: the task tables and exchange plans each
rank would launch, no launches and no collectives)."""

import random

import numpy as np
import torch
import pytest

import cubed_amd as cubed
import cubed_amd.array_api as xp
import cubed_amd.random as crandom
from cubed_amd.core.plan import arrays_to_plan
import cubed_amd._native as nat
import cubed_amd.lowering as Lw
from cubed_amd.lowering import MODE_PARTIALS, MODE_STREAM, FusedLaunch
from cubed_amd.runtime.executors.dist import (
    DistPiecesLaunch,
    FetchLaunch,
    PartialsLaunch,
    RechunkLaunch,
)
from dryrun import DryExecutor, FakeComm


def _quad(dry, T=80):
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    random.seed(1)
    u = xp.astype(crandom.random((T, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    v = xp.astype(crandom.random((T, 16, 32), chunks=(10, 16, 32), spec=spec), xp.float32)
    arrays_to_plan(u, v).execute(executor=dry, array_names=[u.name, v.name])
    dry.launched.clear()
    m = xp.mean(u * v, axis=0)
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    return u, v, m


@pytest.mark.parametrize("world", [2, 3, 8])
def test_quad_means_partials_per_rank(built, world):
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        u, v, m = _quad(dry)
        kinds = [type(l).__name__ for l in dry.launched]
        assert kinds == ["FusedLaunch", "PartialsLaunch"], kinds
        fused, part = dry.launched
        P = fused.prog
        assert P.mode & MODE_PARTIALS and P.mode & MODE_STREAM
        # this rank's share of the 8 time chunks, read in place (slot stride)
        mine = len([c for c in range(8) if c % world == rank])
        assert fused.ntasks == 1 and fused.max_red == 10 * mine or (mine == 0 and fused.max_red == 1)
        assert part.sum_only and part.root == 0 and part.finish_here == (rank == 0)
        assert u.zarray.local_nslots() == mine
        # mean's n is the whole reduced extent (T = 80): filled by the host
        # (CUBED_MODE_HOST_COUNT), never reduced across the ranks
        assert P.mode & 128 and part.host_count == [True, False]
        assert (part.field_view(0) == 80).all()


def _partials(dry, m):
    dry.launched.clear()
    arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
    part = [l for l in dry.launched if isinstance(l, PartialsLaunch)]
    return part[0] if part else None


@pytest.mark.parametrize("world", [2, 3])
def test_host_count_from_geometry_transposed(built, world):
    """mean over axis 0 of a TRANSPOSED non-square input (permute_dims fuses
    into the chain with permuted leaf axes): the host-filled count is the
    reduced extent of the chain's own iteration space (60), not of the leaf
    array's first axis (40) -- the same on every rank."""
    x = np.arange(40 * 60, dtype=np.float64).reshape(40, 60)
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="2GB", executor=dry)
        # row chunks of 40: the chain reads the permuted chunks in place
        a = cubed.from_array(x, chunks=(40, 15), spec=spec)
        arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
        part = _partials(dry, xp.mean(xp.permute_dims(a, (1, 0)), axis=0))
        assert part is not None and part.host_count == [True, False]
        assert (part.field_view(0) == 60).all()


@pytest.mark.parametrize("world", [2, 3])
def test_host_count_from_geometry_broadcast(built, world):
    """mean(u * w, axis=0) with w (16, 32) broadcast against u (80, 16, 32):
    the broadcast leaf has no reduced axis; the count is 80."""
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
        random.seed(2)
        u = crandom.random((80, 16, 32), chunks=(10, 16, 32), spec=spec)
        w = crandom.random((16, 32), chunks=(16, 32), spec=spec)
        arrays_to_plan(u, w).execute(executor=dry, array_names=[u.name, w.name])
        part = _partials(dry, xp.mean(u * w, axis=0))
        assert part is not None and part.host_count == [True, False]
        assert (part.field_view(0) == 80).all()


def test_host_count_geometry_counts_contributing_tasks(built):
    """The geometry count sums every contributing task's reduced extent
    (all ranks), with an edge chunk along the reduced axis (T = 75)."""
    world = 2
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        u, v, m = _quad(dry, T=75)
        part = [l for l in dry.launched if isinstance(l, PartialsLaunch)]
        if part and any(part[0].host_count):
            assert (part[0].field_view(part[0].host_count.index(True)) == 75).all()
        else:  # the edge chunk splits the chain: the count is reduced over the ranks
            assert not part or not any(part[0].host_count)


def test_rechunk_is_one_exchange_per_rank(built):
    world = 4
    x = np.arange(60 * 50, dtype=np.float32).reshape(60, 50)
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem=10**9, executor=dry)
        a = cubed.from_array(x, chunks=(10, 50), spec=spec)
        b = a.rechunk((60, 10))
        arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
        dry.launched.clear()
        arrays_to_plan(b).execute(executor=dry, resume=True, array_names=[b.name])
        rl = [l for l in dry.launched if isinstance(l, RechunkLaunch)]
        assert len(rl) == 1
        plan = rl[0].plan
        # 6 source x 5 target chunks: 10x10 f32 pieces, each a contiguous
        # row band of its (60, 10) target chunk: received in place, no unpack
        assert plan.stage_bytes == 0 and rl[0].unpack.nboxes == 0
        assert plan.pack_bytes == sum(512 for d in range(world) for _ in plan.send[d])
        assert sum(s[0].nboxes for s in rl[0].slices) == sum(len(l) for l in plan.send)
        assert rl[0].local.nboxes == len(plan.local)


def test_misaligned_elementwise_fetches(built):
    world = 2
    y = np.ones((60, 50), dtype=np.float32)
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem=10**9, executor=dry)
        p = cubed.from_array(y, chunks=(10, 50), spec=spec)
        q = cubed.from_array(y, chunks=(10, 50), spec=spec)
        arrays_to_plan(p, q).execute(executor=dry, array_names=[p.name, q.name])
        dry.launched.clear()
        s = p + q  # same grid: no fetch
        arrays_to_plan(s).execute(executor=dry, resume=True, array_names=[s.name])
        assert not [l for l in dry.launched if isinstance(l, FetchLaunch)]
        f = [l for l in dry.launched if isinstance(l, FusedLaunch)]
        assert f and f[0].ntasks == 3  # 6 chunks, block-cyclic over 2 ranks


def test_max_uses_gather_combine(built):
    world = 2
    x = np.random.default_rng(0).random((40, 64))
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="2GB", executor=dry)
        a = cubed.from_array(x, chunks=(10, 64), spec=spec)
        arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
        dry.launched.clear()
        m = xp.max(a, axis=0)
        arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
        part = [l for l in dry.launched if isinstance(l, PartialsLaunch)]
        assert part and not part[0].sum_only


# ------------------------------------------------ collective order agreement


def _launch_sequence(rank, world):
    """Lower a mixed program on this rank (lowering-time agreement runs over
    the real gloo group) and return the sequence of cross-rank launches."""
    from cubed_amd.runtime.comm import Comm

    dry = DryExecutor(Comm())
    spec = cubed.Spec(allowed_mem="2GB", reserved_mem="100MB", executor=dry)
    seq = []

    def go(*arrs, resume=None):
        dry.launched.clear()
        arrays_to_plan(*arrs).execute(executor=dry, resume=resume, array_names=[a.name for a in arrs])
        seq.append([type(l).__name__ for l in dry.launched
                    if isinstance(l, (FetchLaunch, RechunkLaunch, PartialsLaunch, DistPiecesLaunch))])

    random.seed(4)
    u = xp.astype(crandom.random((60, 24, 40), chunks=(10, 24, 40), spec=spec), xp.float32)
    v = xp.astype(crandom.random((60, 24, 40), chunks=(10, 24, 40), spec=spec), xp.float32)
    go(u, v)
    go(xp.mean(u * v, axis=0), resume=True)
    a = crandom.random((200, 200), chunks=(50, 50), spec=spec)
    go(xp.mean((a + 1) * 2, axis=0))
    x = np.random.default_rng(8).random((33, 500)) + 0.5
    b = cubed.from_array(x, chunks=(10, 128), spec=spec)
    go(xp.max(b, axis=0))
    go(xp.min(b))
    go(xp.sum(b, axis=1))  # edge chunk along the reduced axis on one rank only
    y = np.ones((60, 50), dtype=np.float32)
    go(cubed.from_array(y, chunks=(7, 9), spec=spec).rechunk((13, 4)))
    go(cubed.from_array(y, chunks=(10, 50), spec=spec) + cubed.from_array(y, chunks=(20, 25), spec=spec))
    go(xp.mean(cubed.from_array(y, chunks=(7, 50), spec=spec).rechunk((60, 9)), axis=0))
    A = cubed.from_array(np.ones((96, 80), np.float32), chunks=(32, 40), spec=spec)
    B = cubed.from_array(np.ones((80, 64), np.float32), chunks=(40, 32), spec=spec)
    go(xp.matmul(A, B))
    return seq


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_issue_the_same_collectives(built, world):
    from distutil import run_ranks

    seqs = run_ranks(_launch_sequence, world)
    for r in range(1, world):
        assert seqs[r] == seqs[0], (r, seqs[0], seqs[r])
    assert ["PartialsLaunch"] in seqs[0] and ["FetchLaunch"] in seqs[0]


@pytest.mark.parametrize("merge", [False, True])
def test_rechunk_mean_runs_pieces_where_chunks_live(built, monkeypatch, merge):
    """rechunk rows -> columns read through by mean(axis=0) on 4 ranks: each
    rank runs only the pieces of the source chunks it holds (no fetch, no
    all-to-all), one partials row per piece plus an identity row for groups
    without local pieces.  With row merging (the default) a rank's pieces of
    one output block -- its row bands, consecutive slots of its slab -- are
    one row."""
    import cubed_amd.lowering as Lw

    monkeypatch.setattr(Lw, "MERGE_ROWS", merge)
    world = 4
    x = np.ones((500, 500), dtype=np.float32)
    total = 0
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="288GB", executor=dry)
        a = cubed.from_array(x, chunks=(10, 500), spec=spec)
        arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
        dry.launched.clear()
        m = xp.mean(a.rechunk((500, 10)), axis=0)
        arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
        kinds = [type(l).__name__ for l in dry.launched]
        assert kinds == ["DistPiecesLaunch"], kinds
        dp = dry.launched[0]
        assert dp.ngroups == 50 and dp.root is None
        mine = len([c for c in range(50) if c % world == rank])  # source chunks held here
        assert dp.fused.ntasks == (mine * 50 if not merge else 50)
        rows = sum(r.extent[0] for r in dp.fused.layout.rows)
        assert rows == mine * 10 * 50  # every local source row once per output block
        total += dp.fused.ntasks
    assert total == (50 * 50 if not merge else 50 * world)


def test_scatter_owners_are_per_group_when_pieces_cut_a_kept_dim(built):
    """Source chunks (10, 7) rechunked to (500, 10) columns: every target
    column block straddles two source column chunks, so a key has SEVERAL
    groups (one per kept interval).  The combine's owner list is per group
    (the owner of the group's key): the reduce-scatter permutation, the host
    counts and the finish rows all follow it (a per-key list would slice the
    partials at the wrong field stride)."""
    world = 4
    x = np.ones((500, 500), dtype=np.float32)
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="288GB", executor=dry)
        a = cubed.from_array(x, chunks=(10, 7), spec=spec)
        arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
        dry.launched.clear()
        m = xp.mean(a.rechunk((500, 10)), axis=0)
        arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
        dps = [l for l in dry.launched if isinstance(l, DistPiecesLaunch)]
        assert len(dps) == 1
        dp = dps[0]
        nkeys = m.zarray.numblocks[0]
        assert dp.ngroups > nkeys  # pieces cut the kept dim
        sc = dp.scatter
        assert sc is not None and sc.G == dp.ngroups
        # several groups per key (owners are not g mod W): the box-copy permute stays
        assert sc.permute is not None and not dp.fused.prog.mode & Lw.MODE_OWNER_MAJOR
        # each group's owner is its key's owner, and the groups of one key are
        # consecutive: owner-major slots of this rank = its keys' groups
        tbl = sc.dst.view(sc.f1 - sc.f0, sc.G)[0].tolist()
        owner_of = [t // ((sc.f1 - sc.f0) * sc.L) for t in tbl]
        assert sorted(set(owner_of)) == sorted({k % world for k in range(nkeys)})
        mine = [g for g in range(sc.G) if owner_of[g] == rank]
        assert sc.mine == mine
        # every group of this rank is counted over all 500 rows
        cnt = sc.fin.view(torch.int64)[:sc.L * sc.mko].view(sc.L, sc.mko)[:len(mine), 0]
        assert (cnt == 500).all()


def test_rechunk_mean_combines_by_reduce_scatter(built):
    """Several owners of the output blocks: the group partials combine by
    ONE reduce-scatter in owner-major order (each rank receives only its own
    blocks' sums and finishes them), not an all-reduce of every block."""
    world = 4
    x = np.ones((500, 500), dtype=np.float32)
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="288GB", executor=dry)
        a = cubed.from_array(x, chunks=(10, 500), spec=spec)
        arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
        dry.launched.clear()
        m = xp.mean(a.rechunk((500, 10)), axis=0)
        arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
        dp = dry.launched[0]
        sc = dp.scatter
        assert sc is not None and sc.L == 13 and sc.mine == [g for g in range(50) if g % world == rank]
        assert (sc.f0, sc.f1) == (1, 2)  # n is host-filled; only the totals cross the ranks
        assert sc.perm.numel() == world * 13 * 10
        # 10-wide blocks are no streaming program: the box-copy permute stays
        assert sc.permute is not None and not dp.fused.prog.mode & Lw.MODE_OWNER_MAJOR
        cnt = sc.fin.view(torch.int64)[:13 * 10].view(13, 10)
        k = len(sc.mine)  # the counts of this rank's blocks, then padding slots
        assert (cnt[:k] == 500).all() and (cnt[k:] == 1).all()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_stream_partials_write_owner_major(built, world):
    """A streaming partials program with one summed field and block-cyclic
    owners writes its SoA partials straight into the reduce-scatter's
    owner-major order (CUBED_MODE_OWNER_MAJOR; mko, W, L in the last three
    const slots): no box-copy permute, the reduce-scatter reads the SoA block."""
    x = np.ones((500, 512), dtype=np.float32)
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="288GB", executor=dry)
        a = cubed.from_array(x, chunks=(10, 512), spec=spec)
        arrays_to_plan(a).execute(executor=dry, array_names=[a.name])
        dry.launched.clear()
        m = xp.mean(a.rechunk((500, 16)), axis=0)
        arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
        (dp,) = [l for l in dry.launched if isinstance(l, DistPiecesLaunch)]
        sc, P = dp.scatter, dp.fused.prog
        L = -(-32 // world)
        assert dp.soa_direct and sc.L == L and sc.mine == [g for g in range(32) if g % world == rank]
        assert sc.permute is None and P.mode & Lw.MODE_OWNER_MAJOR and P.mode & MODE_STREAM
        assert [P.consts[nat.MAX_CONSTS - i].i for i in (3, 2, 1)] == [16, world, L]
        assert sc.perm.data_ptr() == dp.gsoa.data_ptr() and sc.perm.numel() == world * L * 16
        # the JIT module was rebuilt for the changed program
        if dp.fused.handle is not None:
            assert "cubed_stream" in nat.program_source(dp.fused.handle)


# ------------------------------------------------ multi-GPU matmul (packed A image)


def _matmul_dry(rank, world, dtype, shape=(700, 1600, 2048), chunks=(300, 200, 264)):
    from cubed_amd.runtime.executors.dist import DistGemmLaunch

    M, K, N = shape
    dry = DryExecutor(FakeComm(rank, world))
    spec = cubed.Spec(allowed_mem="288GB", executor=dry)
    random.seed(3)
    A = xp.astype(crandom.random((M, K), chunks=(chunks[0], chunks[1]), spec=spec), dtype)
    B = xp.astype(crandom.random((K, N), chunks=(chunks[1], chunks[2]), spec=spec), dtype)
    arrays_to_plan(A, B).execute(executor=dry, array_names=[A.name, B.name])
    dry.launched.clear()
    C = xp.matmul(A, B)
    arrays_to_plan(C).execute(executor=dry, resume=True, array_names=[C.name])
    return [l for l in dry.launched if isinstance(l, DistGemmLaunch)], dry.launched


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_matmul_packs_and_exchanges_the_a_image(built, world, dtype):
    """Config 5's shape of work (8 x 8 chunk grid), reduced: every rank packs
    the k blocks starting in its own A chunks into the k-major image, sends
    each owned block run to every peer and receives the others' in place;
    the block ranges tile the image exactly, halos reach < one block into
    the next chunk, and every transfer pairs with the peer's."""
    dt = xp.bfloat16 if dtype == "bfloat16" else xp.float32
    T = 64 if dtype == "bfloat16" else 16
    launches = [_matmul_dry(r, world, dt) for r in range(world)]
    plans = []
    for r, (dg, all_l) in enumerate(launches):
        assert len(dg) == 1 and [type(l).__name__ for l in all_l] == ["DistGemmLaunch"]
        d = dg[0]
        plans.append(d)
        assert d.K == 1600 and d.KTL == -(-1600 // T) and d.TM == 3
        cover = sorted(x for q in range(8) for x in range(*d.ranges[q]))
        assert cover == list(range(d.KTL))
        for q in range(7):
            assert 0 <= d.halo_w[q] < T and (200 * (q + 1) + d.halo_w[q]) % T == 0
        assert d.owned == [q for q in range(8) if q % world == r]
        assert d.tj == 8 // world and d.ti == 3
        assert d.bytes_out == (world - 1) * d.own_bytes[r]
        assert d.bytes_in == sum(d.own_bytes[p] for p in range(world) if p != r)
    # transfers pair up: per (sender, receiver) the same sizes in the same order
    for s in range(world):
        for p in range(world):
            if s == p:
                continue
            sent = [v.numel() for v, peer in plans[s].region_sends if peer == p]
            got = [v.numel() for v, peer in plans[p].region_recvs if peer == s]
            assert sent == got and sent
            hs = [v.numel() for v, peer in plans[s].halo_sends if peer == p]
            hr = [v.numel() for v, peer in plans[p].halo_recvs if peer == s]
            assert hs == hr


def test_matmul_off_the_regular_ownership_fetches_chunks(built):
    """3 ranks do not divide an 8 x 8 chunk grid: the whole-chunk fetch path
    (FetchLaunch + the chained GEMM) runs instead."""
    dg, all_l = _matmul_dry(0, 3, xp.float32)
    assert not dg and "FetchLaunch" in [type(l).__name__ for l in all_l]


@pytest.mark.parametrize("world", [2, 3])
def test_oversized_program_splits_on_every_rank(built, world):
    """A chunk function over five inputs is split into HBM temporaries on
    several GPUs too: each temporary is block-cyclic like the task space, so
    every rank computes and reads only the chunks of its own tasks; the
    reduction over several chunks per output block then combines across
    ranks as usual."""
    for rank in range(world):
        dry = DryExecutor(FakeComm(rank, world))
        spec = cubed.Spec(allowed_mem="2GB", executor=dry)
        random.seed(21)
        five = [crandom.random((60, 40), chunks=(10, 20), spec=spec) for _ in range(5)]
        arrays_to_plan(*five).execute(executor=dry, array_names=[a.name for a in five])
        dry.launched.clear()
        y5 = cubed.map_blocks(lambda a, b, c, d, e: a * b + c * d - e, *five, dtype=np.float64)
        m = xp.mean(y5, axis=0)
        arrays_to_plan(m).execute(executor=dry, resume=True, array_names=[m.name])
        kinds = [type(l).__name__ for l in dry.launched]
        assert kinds.count("FusedLaunch") >= 2 and kinds[-1] in ("DistPiecesLaunch", "PartialsLaunch"), kinds
        mine = [c for c in range(12) if c % world == rank]  # 6 x 2 chunk grid, block-cyclic
        split = [l for l in dry.launched if isinstance(l, FusedLaunch)]
        assert all(l.ntasks <= len(mine) for l in split)

"""runtime.comm.LoopbackComm on CPU tensors: the rehearsal comm keeps the
Comm interface the executor calls, copies the bytes a collective would move
on this rank's side, records reduce inputs, and never combines values."""

import pytest
import torch

from cubed_amd.runtime.comm import LoopbackComm


def test_rank_checked():
    with pytest.raises(ValueError):
        LoopbackComm(8, 8)
    c = LoopbackComm(3, 8)
    assert (c.rank, c.world) == (3, 8)
    assert c.all_ok(True) and not c.all_ok(False)


def test_reduce_records_and_keeps_values():
    c = LoopbackComm(1, 4, record=True)
    t = torch.arange(10, dtype=torch.float64)
    c.all_reduce_sum(t)
    c.reduce_sum(t * 2, 0)
    assert torch.equal(t, torch.arange(10, dtype=torch.float64))  # not summed over ranks
    kinds = [k for k, _ in c.records]
    assert kinds == ["all_reduce_sum", "reduce_sum"]
    assert torch.equal(c.records[1][1], torch.arange(10, dtype=torch.float64) * 2)
    t.add_(1)
    assert c.records[0][1][0] == 0  # a copy, not a view


def test_all_gather_fills_every_slot():
    c = LoopbackComm(0, 3)
    t = torch.tensor([1, 2], dtype=torch.int64)
    out = torch.zeros(6, dtype=torch.int64)
    c.all_gather(out, t)
    assert out.tolist() == [1, 2, 1, 2, 1, 2]


def test_skip_collectives_moves_nothing():
    """Timing mode: the collectives touch no buffer (records still kept)."""
    c = LoopbackComm(2, 4, record=True)
    c.skip_collectives = True
    t = torch.arange(8, dtype=torch.float64)
    out = torch.full((2,), -1.0, dtype=torch.float64)
    c.reduce_scatter_sum(out, t)
    g = torch.zeros(24, dtype=torch.float64)
    c.all_gather(g, t)
    c.all_reduce_sum(t)
    c.broadcast(t, 0)
    assert out.tolist() == [-1.0, -1.0] and not g.any()
    assert c._scratch is None
    assert [k for k, _ in c.records] == ["reduce_scatter_sum", "all_reduce_sum"]
    c.skip_collectives = False
    c.reduce_scatter_sum(out, t)
    assert out.tolist() == [4.0, 5.0]


def test_exchange_alone_writes_every_receive():
    """Without a mesh a rehearsed rank writes each receive (from scratch:
    the arriving bytes' write traffic) and reads nothing of its sends into
    them -- the round-4 form paired sends with receives by list position."""
    c = LoopbackComm(2, 8)
    s = [(torch.arange(4, dtype=torch.uint8), 1), (torch.arange(4, 8, dtype=torch.uint8), 3)]
    r = [(torch.full((6,), 7, dtype=torch.uint8), 5)]
    c.exchange(s, r).wait()
    assert (c.sent_bytes, c.recv_bytes) == (8, 6)
    with pytest.raises(ValueError):
        c.exchange([(s[0][0], 2)], [])  # to itself
    send = torch.arange(6, dtype=torch.uint8)
    recv = torch.zeros(8, dtype=torch.uint8)
    c.all_to_all(recv, send, [3, 3], [3, 3])
    assert recv[:6].tolist() == list(range(6))


def test_mesh_matches_transfers_by_peer_and_order():
    """Three rehearsed ranks: the receives of the replay phase get the bytes
    the PEER sent, pair by pair in issue order, whatever the order of the
    receive list across peers."""
    from cubed_amd.runtime.comm import LoopbackMesh

    mesh = LoopbackMesh(3)
    comms = [LoopbackComm(r, 3, mesh=mesh) for r in range(3)]

    def t(*v):
        return torch.tensor(v, dtype=torch.uint8)

    sends = {0: [(t(1, 2), 1), (t(3, 4, 5), 2), (t(6), 1)],
             1: [(t(10, 11, 12), 2), (t(13), 0)],
             2: [(t(20), 0), (t(21, 22), 1)]}
    shapes = {0: [(1, 1), (2, 1)], 1: [(0, 2), (2, 2), (0, 1)], 2: [(1, 3), (0, 3)]}

    def recvs(r):
        return [(torch.zeros(n, dtype=torch.uint8), peer) for peer, n in shapes[r]]

    for r in range(3):  # record: receives untouched
        comms[r].exchange(sends[r], recvs(r))
    assert mesh.bytes_between(0, 1) == 3 and mesh.bytes_between(1, 2) == 3
    mesh.phase = "replay"
    got = {}
    for step in range(2):  # the cursors wrap: every step sees the same bytes
        for r in range(3):
            rv = recvs(r)
            comms[r].exchange(sends[r], rv)
            got[r] = [x.tolist() for x, _ in rv]
        assert got[0] == [[13], [20]]
        assert got[1] == [[1, 2], [21, 22], [6]]
        assert got[2] == [[10, 11, 12], [3, 4, 5]]
    bad = [(torch.zeros(5, dtype=torch.uint8), 1)]
    with pytest.raises(RuntimeError, match="B, the receive"):
        comms[0].exchange([], bad)


def test_mesh_collectives_combine_every_rank():
    """With a LoopbackMesh the collectives of rehearsed ranks are matched by
    issue index: a replay pass combines ALL ranks' inputs (sums in rank
    order), so a multi-rank reduction or all-gather rehearsed in one process
    gives every rank what RCCL would."""
    from cubed_amd.runtime.comm import LoopbackMesh

    W = 3
    mesh = LoopbackMesh(W)
    comms = [LoopbackComm(r, W, mesh=mesh) for r in range(W)]

    def step(r):
        c = comms[r]
        a = torch.arange(6, dtype=torch.float64) + 10 * r
        c.all_reduce_sum(a)
        red = torch.full((2,), float(r + 1), dtype=torch.float64)
        c.reduce_sum(red, 1)
        rs_in = torch.arange(W * 2, dtype=torch.int64) * (r + 1)
        rs_out = torch.zeros(2, dtype=torch.int64)
        c.reduce_scatter_sum(rs_out, rs_in)
        g = torch.zeros(W * 2, dtype=torch.int64)
        c.all_gather(g, torch.tensor([r, -r], dtype=torch.int64))
        b = torch.tensor([r * 7], dtype=torch.int64)
        c.broadcast(b, 2)
        # all-to-all: rank r sends r+1 bytes of value 10r + q to rank q
        ss = [r + 1] * W
        send = torch.cat([torch.full((r + 1,), 10 * r + q, dtype=torch.uint8) for q in range(W)])
        rsp = [q + 1 for q in range(W)]
        recv = torch.zeros(sum(rsp), dtype=torch.uint8)
        c.all_to_all(recv, send, rsp, ss)
        return a, red, rs_out, g, b, recv

    for r in range(W):
        step(r)
    mesh.phase = "replay"
    for _ in range(2):
        for r in range(W):
            a, red, rs_out, g, b, recv = step(r)
            assert a.tolist() == [3 * i + 30 for i in range(6)]
            assert red.tolist() == ([6.0, 6.0] if r == 1 else [float(r + 1)] * 2)
            assert rs_out.tolist() == [6 * (2 * r), 6 * (2 * r + 1)]
            assert g.tolist() == [0, 0, 1, -1, 2, -2]
            assert b.tolist() == [14]
            want = []
            for q in range(W):
                want += [10 * q + r] * (q + 1)
            assert recv.tolist() == want


def test_mesh_replay_refreshes_sends_that_depend_on_receives():
    """A send whose bytes come from an earlier receive (a halo received,
    then forwarded) is right after a second replay pass: replayed sends
    overwrite what the record pass kept."""
    from cubed_amd.runtime.comm import LoopbackMesh

    mesh = LoopbackMesh(2)
    comms = [LoopbackComm(r, 2, mesh=mesh) for r in range(2)]
    own = [torch.tensor([5], dtype=torch.uint8), torch.tensor([9], dtype=torch.uint8)]
    got = {}

    def step(r):
        c = comms[r]
        halo = torch.zeros(1, dtype=torch.uint8)
        c.exchange([(own[r], 1 - r)], [(halo, 1 - r)])
        fwd = own[r] + halo  # depends on the receive
        out = torch.zeros(1, dtype=torch.uint8)
        c.exchange([(fwd, 1 - r)], [(out, 1 - r)])
        got[r] = out.item()

    for r in range(2):
        step(r)
    mesh.phase = "replay"
    for _ in range(2):
        for r in range(2):
            step(r)
    assert got == {0: 14, 1: 14}

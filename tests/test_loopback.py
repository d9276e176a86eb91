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


def test_exchange_and_all_to_all_copy_bytes():
    c = LoopbackComm(2, 8)
    s = [(torch.arange(4, dtype=torch.uint8), 1), (torch.arange(4, 8, dtype=torch.uint8), 3)]
    r = [(torch.zeros(4, dtype=torch.uint8), 1), (torch.zeros(4, dtype=torch.uint8), 3)]
    c.exchange(s, r).wait()
    assert r[0][0].tolist() == [0, 1, 2, 3] and r[1][0].tolist() == [4, 5, 6, 7]
    send = torch.arange(6, dtype=torch.uint8)
    recv = torch.zeros(8, dtype=torch.uint8)
    c.all_to_all(recv, send, [3, 3], [3, 3])
    assert recv[:6].tolist() == list(range(6))

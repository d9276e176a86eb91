"""bench.py's multi-GPU launch contract (CPU, no GPU touched).

The driver runs ``python bench.py --gpus N`` (and, for N > 1, sometimes
under torch.distributed.run itself).  Outside torchrun, --gpus N > 1 must
re-launch N ranks as a child process before any GPU call; under torchrun,
WORLD_SIZE must match --gpus or the run fails instead of timing the wrong
number of GPUs."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_command_is_torchrun_with_n_ranks():
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "5"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_gpus_n_relaunches_before_touching_the_gpu(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: calls.append(cmd) or 0)
    monkeypatch.setattr(bench, "setup_dist", lambda a: pytest.fail("touched the GPU in the parent"))
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "4", "--steps", "3"])
    assert e.value.code == 0
    assert len(calls) == 1 and "--nproc-per-node=4" in calls[0]
    assert calls[0][-4:] == ["--gpus", "4", "--steps", "3"]


def test_child_status_is_propagated(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: 7)
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2"])
    assert e.value.code == 7


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "8"])
    assert e.value.code == 2


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: pytest.fail("relaunched for --gpus 1"))
    args = bench.parse(["--gpus", "1"])
    bench.maybe_relaunch(args, ["--gpus", "1"])  # returns: runs here


def test_extras_selection():
    assert set(bench.EXTRAS) >= {"rechunk", "rechunk_mean", "config1", "vorticity", "matmul_f32",
                                 "matmul_bf16"}

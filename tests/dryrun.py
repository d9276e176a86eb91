"""Lower-only executor for CPU tests (test infrastructure, not a CPU path).

``DryExecutor`` runs the MI355X executor's lowering on a CPU "device": plans
are lowered to the exact kernel-argument tables the GPU path would launch, but
no launch runs (and nothing is computed), so tests can check task tables,
fusion decisions and launch counts without a GPU.
"""

import torch

import cubed_amd.lowering as L
import cubed_amd.runtime.executors.gpu as g


class FakeComm:
    """Rank/world of a multi-GPU executor for lowering-only tests; any
    collective call is an error (dry runs launch nothing)."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world

    def all_ok(self, ok):
        return ok

    def __getattr__(self, name):
        raise AssertionError(f"dry run called the collective {name}")


class DryExecutor(g.GpuDagExecutor):
    def __init__(self, comm=None):
        self._init_state(torch.device("cpu"), 0, True)
        self.set_comm(comm)
        self.launched = []

    @property
    def stream(self):
        return 0

    def execute_dag(self, *args, **kwargs):
        import cubed_amd.runtime.executors.dist as D

        saved = {}
        for cls in (L.FusedLaunch, L.CopyLaunch, L.GemmLaunch, D.FetchLaunch, D.RechunkLaunch,
                    D.PartialsLaunch, D.DistPiecesLaunch, D.DistGemmLaunch):
            saved[cls] = cls.run
            cls.run = lambda launch, stream, _log=self.launched: _log.append(launch)
        try:
            return super().execute_dag(*args, **kwargs)
        finally:
            for cls, fn in saved.items():
                cls.run = fn

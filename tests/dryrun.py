"""Lower-only executor for CPU tests (test infrastructure, not a CPU path).

``DryExecutor`` runs the MI355X executor's lowering on a CPU "device": plans
are lowered to the exact kernel-argument tables the GPU path would launch, but
no launch runs (and nothing is computed), so tests can check task tables,
fusion decisions and launch counts without a GPU.
"""

import torch

import cubed_amd.lowering as L
import cubed_amd.runtime.executors.gpu as g


class DryExecutor(g.GpuDagExecutor):
    def __init__(self):
        self._init_state(torch.device("cpu"), 0, True)
        self.launched = []

    @property
    def stream(self):
        return 0

    def execute_dag(self, *args, **kwargs):
        saved = {}
        for cls in (L.FusedLaunch, L.CopyLaunch, L.GemmLaunch):
            saved[cls] = cls.run
            cls.run = lambda launch, stream, _log=self.launched: _log.append(launch)
        try:
            return super().execute_dag(*args, **kwargs)
        finally:
            for cls, fn in saved.items():
                cls.run = fn

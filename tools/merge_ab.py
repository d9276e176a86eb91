"""A/B of the executor's task-row merging (lowering.MERGE_ROWS): runs bench.py
in this process with merging off or on.  Development aid.
    python tools/merge_ab.py off|rows|on [bench.py args]   (rows: group rows only, no kept-dim merge)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import cubed_amd.lowering as L  # noqa: E402

L.MERGE_ROWS = sys.argv[1] in ("on", "rows")
L.MERGE_KEPT = sys.argv[1] == "on"
import bench  # noqa: E402

bench.main(sys.argv[2:])

"""A/B of a patched streaming kernel body: the JIT pointed at a copy of
csrc/ whose kernels.h carries the arm's patch.  Development aid.
    python tools/stream_patch_ab.py base|xcd [bench.py args]
xcd: workgroup g -> logical (g % 8) * (G / 8) + g / 8, so the 8 XCDs (round-robin
dispatch) each run one contiguous run of (task, split, column block) -- the
column blocks either side of a line a misaligned row splits share an L2."""
import os
import shutil
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cubed_amd import _native as nat  # noqa: E402

PATCHES = {
    "xcd": ("  const int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;\n  const int64_t b = g % bpt;",
            "  const int64_t G = (int64_t)gridDim.x * gridDim.y;\n"
            "  int64_t g = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;\n"
            "  if ((G & 7) == 0) g = (g & 7) * (G >> 3) + (g >> 3);\n"
            "  const int64_t b = g % bpt;"),
}

arm = sys.argv[1]
if arm in PATCHES:
    src = os.path.join(os.path.dirname(nat.__file__), "csrc")
    dst = os.path.join(tempfile.mkdtemp(), "csrc")
    shutil.copytree(src, dst)
    p = os.path.join(dst, "kernels.h")
    s = open(p).read()
    old, new = PATCHES[arm]
    i = s.index("CUBED_DEV void stream_body(")
    j = s.index(old, i)
    s = s[:j] + new + s[j + len(old):]
    open(p, "w").write(s)
    nat.INCLUDE_DIRS = ";".join([dst] + nat.INCLUDE_DIRS.split(";")[1:])
import bench  # noqa: E402

bench.main(sys.argv[2:])

"""A/B of the streaming kernels' load form: non-temporal (the library's
kernels.h) vs cached 16-B loads, by pointing the JIT at a patched copy of
csrc/ (kernels.h with cached ld4 / CUBED_LD64_CACHED).  Development aid.
    python tools/ld_ab.py nt|cached [bench.py args]"""
import os
import shutil
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cubed_amd import _native as nat  # noqa: E402

if sys.argv[1] == "cached":
    src = os.path.join(os.path.dirname(nat.__file__), "csrc")
    dst = os.path.join(tempfile.mkdtemp(), "csrc")
    shutil.copytree(src, dst)
    p = os.path.join(dst, "kernels.h")
    s = open(p).read()
    old = "  const f32x4 v = __builtin_nontemporal_load((const CUBED_G f32x4*)p);\n  o[0] = v.x;"
    assert old in s
    s = s.replace(old, "  const f32x4 v = *(const CUBED_G f32x4*)p;\n  o[0] = v.x;", 1)
    old = "  const f64x2 a = __builtin_nontemporal_load((const CUBED_G f64x2*)p);\n  const f64x2 b = __builtin_nontemporal_load((const CUBED_G f64x2*)(p + 2));"
    assert old in s
    s = s.replace(old, "  const f64x2 a = *(const CUBED_G f64x2*)p;\n  const f64x2 b = *(const CUBED_G f64x2*)(p + 2);", 1)
    s = "#define CUBED_LD64_CACHED 1\n" + s
    open(p, "w").write(s)
    nat.INCLUDE_DIRS = ";".join([dst] + nat.INCLUDE_DIRS.split(";")[1:])
import bench  # noqa: E402

bench.main(sys.argv[2:])

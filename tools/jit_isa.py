"""Compile the streaming JIT kernels of a few representative mean programs
offline (hipcc, no GPU) and report their register use, scratch and LDS --
a check that a kernel-body change did not push the specialised kernels into
scratch (development aid; the product compiles the same source with hipRTC).

    python tools/jit_isa.py [--keep DIR]
"""
import argparse
import ctypes
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cubed_amd import _native as nat  # noqa: E402
from cubed_amd import ir  # noqa: E402
from cubed_amd.lowering import (LEAF_ARRAY, MODE_PARTIALS, MODE_STREAM, MODE_STREAM_W2,  # noqa: E402
                                V_F32, V_F64, _OPCODES)

OPS = dict(_OPCODES)
OPS.update({k: v for k, v in ir.BINARY_OPS.items()})


def mean_program(vtype, nleaves, nred, w_bits=0, partials=False):
    """mean(prod of the leaves) over nred reduced dims: fields total (SUM f64)
    and n (COUNT), epilogue total / n, f32/f64 output."""
    P = nat.Program()
    P.vtype = vtype
    P.ndim = nred + 1
    P.nred = nred
    P.mode = 4 | MODE_STREAM | w_bits | (MODE_PARTIALS if partials else 0)
    P.nleaves = nleaves
    dt = ir.dtype_code("float32" if vtype == V_F32 else "float64")
    for l in range(nleaves):
        P.leaf_kind[l] = LEAF_ARRAY
        P.leaf_dtype[l] = dt
    n = 0
    for l in range(1, nleaves):  # r0 *= r_l
        I = P.insns[n]
        I.op, I.a, I.b = OPS["multiply"], 0, l
        n += 1
    P.ninsns = n
    P.nfields = 2
    P.field_rop[0], P.field_acc[0], P.field_src[0] = ir.ROPS["sum"], 0, 0
    P.field_rop[1], P.field_acc[1], P.field_src[1] = ir.ROPS["count"], 1, 0
    P.nouts = 1
    P.out_dtype[0] = dt
    P.out_src[0] = 0
    E = P.epi[0]
    E.op, E.a, E.b = OPS["divide"], 0, 1
    P.nepi = 1
    return P


CASES = {
    "quad_means f32 l2 r1 W2": dict(vtype=V_F32, nleaves=2, nred=1, w_bits=MODE_STREAM_W2),
    "share f32 l1 r1 W1": dict(vtype=V_F32, nleaves=1, nred=1),
    "config1 f64 l1 r2 W1": dict(vtype=V_F64, nleaves=1, nred=2),
    "partials f32 l1 r1": dict(vtype=V_F32, nleaves=1, nred=1, partials=True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keep", default=None)
    args = ap.parse_args()
    out = args.keep or tempfile.mkdtemp()
    os.makedirs(out, exist_ok=True)
    inc = nat.INCLUDE_DIRS.split(";")
    for name, kw in CASES.items():
        P = mean_program(**kw)
        h = nat.compile_program(P)  # hipRTC: proves the product compile works
        src = nat.program_source(h)
        tag = re.sub(r"\W+", "_", name)
        path = os.path.join(out, tag + ".hip")
        with open(path, "w") as f:
            f.write(src)
        asm = os.path.join(out, tag + ".s")
        cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-ffp-contract=off", "-DCUBED_JIT=1", "--cuda-device-only", "-S", "-o", asm, path,
               "-Wno-pass-failed"] + [f"-I{d}" for d in inc]
        subprocess.run(cmd, check=True)
        text = open(asm).read()
        stats = {}
        for key in ("vgpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size",
                    "agpr_count"):
            m = re.findall(rf"\.{key}:\s+(\d+)", text)
            stats[key] = m
        spills = re.findall(r"; (?:VGPRs|ScratchSize|Occupancy|NumVgprs|NumSgprs)[^\n]*", text)
        print(f"{name}: code {nat.lib().cubed_fused_code_bytes(h)} B  {stats}")
        for s in spills:
            print("   ", s.strip())


if __name__ == "__main__":
    main()

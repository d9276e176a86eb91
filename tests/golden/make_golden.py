"""Generate the golden fixtures the oracle and the MI355X path are pinned to.

Run in the build container (the reference tree is only present here):
    python tests/golden/make_golden.py

* philox_blocks.json   -- numpy Generator(Philox(key=root_seed + offset)).random()
                          values, i.e. the exact call of cubed/random.py:31-36.
* rechunk_plans.json   -- (read, int, write) chunks from the REFERENCE planner
                          cubed/vendor/rechunker/algorithm.py, imported
                          standalone from /root/reference (it has no zarr
                          dependency), for the BASELINE configs and the
                          reference tests' cases, including its error messages.
* reference_cases.json -- the inline arrays + numpy expectations of the
                          reference's hot-path tests (test_array_api.py,
                          test_core.py, test_nan_functions.py).
Nothing from the reference is copied into the repo: only these inputs and
outputs are stored.
"""
import json
import os
import random
import sys

import numpy as np
from numpy.random import Generator, Philox

HERE = os.path.dirname(os.path.abspath(__file__))


def philox_cases():
    out = []
    random.seed(42)
    rs42 = random.getrandbits(128)
    cases = [(rs42, 0, [8]), (rs42, 1, [3, 5]), (rs42, 15, [7]), (12345, 0, [9]),
             (2**128 - 17, 3, [6]), (2**64 - 1, 1, [5]), (0, 0, [4, 4])]
    for seed, off, shape in cases:
        vals = Generator(Philox(key=seed + off)).random(tuple(shape))
        out.append({"root_seed": str(seed), "offset": off, "shape": shape,
                    "values": [float.hex(float(v)) for v in vals.reshape(-1)]})
    # a long stream: checksum of 1e5 values (exercises counter carry across blocks)
    v = Generator(Philox(key=rs42 + 7)).random(100003)
    out.append({"root_seed": str(rs42), "offset": 7, "shape": [100003],
                "sum": float.hex(float(np.sum(v))), "first": float.hex(float(v[0])),
                "last": float.hex(float(v[-1]))})
    return {"root_seed_after_seed_42": hex(rs42), "cases": out}


def rechunk_cases():
    sys.path.insert(0, "/root/reference/cubed/vendor")
    from rechunker.algorithm import rechunking_plan  # the reference's own planner

    cases = [
        # config 3 at several memory budgets (allowed_mem -> max_mem = allowed//4)
        ((50000, 50000), (1000, 50000), (50000, 1000), 4, 2_000_000_000 // 4),
        ((50000, 50000), (1000, 50000), (50000, 1000), 4, 8_000_000_000 // 4),
        ((50000, 50000), (1000, 50000), (50000, 1000), 4, 288_000_000_000 // 4),
        ((50000, 50000), (500, 50000), (50000, 500), 4, 2_000_000_000 // 4),
        ((50000, 50000), (6250, 50000), (50000, 1000), 4, 2_000_000_000 // 4),
        # reference tests (test_core.py test_rechunk*, primitive/test_rechunk.py)
        ((3, 3), (2, 1), (1, 2), 8, 100000 // 4),
        ((4, 4), (1, 4), (4, 1), 8, (4 * 8 * 4) // 4),
        ((4, 4), (1, 2), (2, 1), 8, 1000 // 4),
        ((8, 8), (2, 8), (8, 2), 8, 800 // 4),
        ((10, 10), (2, 3), (5, 5), 1, 100000 // 4),
        ((20000, 20000), (5000, 5000), (20000, 1000), 8, 2_000_000_000 // 4),
        ((1000, 720, 1440), (10, 720, 1440), (1000, 72, 144), 4, 2_000_000_000 // 4),
    ]
    out = []
    for shape, src, tgt, isz, max_mem in cases:
        rec = {"shape": list(shape), "source_chunks": list(src), "target_chunks": list(tgt),
               "itemsize": isz, "max_mem": max_mem}
        try:
            r, i, w = rechunking_plan(shape, src, tgt, isz, max_mem)
            rec.update(read=list(map(int, r)), int=list(map(int, i)), write=list(map(int, w)))
        except ValueError as e:
            rec["error"] = str(e)
        out.append(rec)
    return out


def reference_cases():
    a33 = [[1, 2, 3], [4, 5, 6], [7, 8, 9]]
    f33 = [[1.0, 2.0, 3.0], [4.0, 5.0, 6.0], [7.0, 8.0, 9.0]]
    m44 = np.arange(1, 17).reshape(4, 4)
    ar = np.arange(242).reshape(11, 22)
    nanx = np.array([[1.0, 2.0, np.nan], [4.0, np.nan, 6.0], [np.nan, 8.0, 9.0]])
    cases = {
        "add": {"a": a33, "b": [[1] * 3] * 3, "chunks": [2, 2],
                "expected": (np.array(a33) + 1).tolist()},
        "mean_axis_0": {"a": f33, "chunks": [2, 2], "expected": np.array(f33).mean(axis=0).tolist()},
        "sum": {"a": a33, "chunks": [2, 2], "expected": int(np.array(a33).sum())},
        "sum_axis_0": {"a": a33, "chunks": [2, 2], "expected": [12, 15, 18]},
        "matmul": {"a": m44.tolist(), "chunks": [2, 2], "expected": (m44 @ m44).tolist()},
        "astype_int32": {"a": a33, "chunks": [2, 2], "expected": a33},
        "negative": {"a": a33, "chunks": [2, 2], "expected": (-np.array(a33)).tolist()},
        "partial_reduce_sum_axis0": {"a_shape": [11, 22], "chunks": [3, 4],
                                     "expected": ar.sum(axis=0, keepdims=True).tolist()},
        "nanmean_all": {"a": [[1.0, 2.0, float("nan")]] + f33[1:], "chunks": [2, 2]},
        "nansum_axis_0": {"a": nanx.tolist(), "chunks": [2, 2],
                          "expected": np.nansum(nanx, axis=0).tolist()},
        "reduction_multiple_rounds_uint8": {"shape": [100, 10], "chunks": [1, 10],
                                            "allowed_mem": 1000,
                                            "expected": np.ones((100, 10)).sum(axis=0).tolist()},
        "tensordot_axes_1": {"x_shape": [20, 20], "y_shape": [20, 10], "x_chunks": [5, 4],
                             "y_chunks": [4, 5],
                             "expected": np.tensordot(np.arange(400).reshape(20, 20),
                                                      np.arange(200).reshape(20, 10), axes=1).tolist()},
    }
    x = np.array([[1.0, 2.0, np.nan]] + f33[1:])
    cases["nanmean_all"]["expected"] = float(np.nanmean(x))
    return cases


def main():
    with open(os.path.join(HERE, "philox_blocks.json"), "w") as f:
        json.dump(philox_cases(), f, indent=1)
    with open(os.path.join(HERE, "rechunk_plans.json"), "w") as f:
        json.dump(rechunk_cases(), f, indent=1)
    with open(os.path.join(HERE, "reference_cases.json"), "w") as f:
        json.dump(reference_cases(), f, indent=1)
    print("wrote golden fixtures")


if __name__ == "__main__":
    main()

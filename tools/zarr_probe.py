"""Zarr v2 source/sink throughput on one GPU (not part of the bench line):
to_zarr of a (4000, 5000) f64 random array in (1000, 5000) chunks (160 MB, 4
chunks of 40 MB) and from_zarr of it back into HBM, per compressor.  Prints
one JSON line with MB/s of array bytes (host codec + pinned transfers)."""
import json
import os
import random
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cubed_amd as cubed  # noqa: E402
import cubed_amd.random as crandom  # noqa: E402
from cubed_amd.runtime.executors.gpu import GpuDagExecutor  # noqa: E402


def main():
    ex = GpuDagExecutor("cuda:0")
    spec = cubed.Spec(allowed_mem="2GB", executor=ex)
    shape, chunks = (16000, 5000), (1000, 5000)
    out = {"shape": shape, "chunks": chunks, "dtype": "f64", "threads": os.cpu_count()}
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for name, comp in (("blosc-lz4", "default"), ("none", None), ("zlib-1", {"id": "zlib", "level": 1})):
            random.seed(1)
            x = crandom.random(shape, chunks=chunks, spec=spec)
            # rounded values compress like real gridded data
            y = x
            path = os.path.join(tmp, name)
            from cubed_amd import zarr_io as Z

            t = Z.open_array(path, mode="w", shape=shape, dtype=np.float64, chunks=chunks, compressor=comp)
            y.compute()  # materialise first: time only the sink
            t0 = time.perf_counter()
            cubed.store(y, t)
            tw = time.perf_counter() - t0
            size = sum(os.path.getsize(os.path.join(path, f)) for f in os.listdir(path))
            z = cubed.from_zarr(path, spec=spec)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            z.compute(_return_in_memory_array=False)
            torch.cuda.synchronize()
            tr = time.perf_counter() - t0
            nb = y.nbytes
            out[name] = {"write_MBps": round(nb / tw / 1e6, 1), "read_MBps": round(nb / tr / 1e6, 1),
                         "ratio": round(nb / size, 3)}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

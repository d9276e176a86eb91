"""Per-launch HBM traffic of the benchmarked kernel from rocprofv3 PMC runs.

Usage (on the GPU box, two separate counter passes, kernel-trace only):
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d OUT/write -o run -- python3 bench.py ...
    python tools/traffic.py OUT/fetch OUT/write KERNEL_NAME > profiles/traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section),
gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
The median over the kernel's dispatches is reported (the first dispatches of
a run can include cold-start effects).
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter, kernel_sub):
    """Counter value per dispatch of the kernel named exactly `kernel_sub`
    (a substring would also pick up its _finalize companion)."""
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if name != kernel_sub or row.get("Counter_Name") != counter:
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(vals))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fetch_dir, write_dir, kernel = sys.argv[1], sys.argv[2], sys.argv[3]
    f = per_dispatch(fetch_dir, "FETCH_SIZE", kernel)
    w = per_dispatch(write_dir, "WRITE_SIZE", kernel)
    out = {"kernel": kernel, "dispatches": [len(f), len(w)]}
    if f:
        out["fetch_bytes"] = 2 * 1024 * statistics.median(f)  # gfx950: FETCH_SIZE = half the bytes
    if w:
        out["write_bytes"] = 1024 * statistics.median(w)
    if f and w:
        out["quad_means_fused"] = out["fetch_bytes"] + out["write_bytes"]
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

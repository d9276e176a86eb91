"""Per-launch HBM traffic of benchmarked kernels from rocprofv3 PMC runs.

Usage (on the GPU box, two separate counter passes, kernel-trace only):
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d OUT/write -o run -- python3 bench.py ...
    python tools/traffic.py OUT/fetch OUT/write KEY=KERNEL [KEY=KERNEL ...] > traffic.json

KERNEL is matched against the dispatched kernel's base name (the name without
"void ", namespaces, template arguments and parameters), exactly; KERNEL@GRID
keeps only dispatches of that grid size (kernels of one name in several
extras, e.g. the elided rechunk + mean and the materialised mean).
FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section),
gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
The median over the kernel's dispatches is reported.

    python tools/traffic.py --compact DIR COUNTER > DIR.json
folds one pass's CSVs (which can exceed what a GPU call brings back) into
{base name: {grid: [value per dispatch]}}; a .json in place of a directory
above is read as such a file.
"""
import csv
import glob
import json
import os
import statistics
import sys


def base_name(name):
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    n = n.split("<")[0].split("(")[0]
    return n.split("::")[-1]


def compact(d, counter):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = base_name(row.get("Kernel_Name") or row.get("Kernel-Name") or "")
                grid = row.get("Grid_Size") or row.get("Grid_Size_X") or ""
                key = (name, grid, path, row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(vals)))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (name, grid, _, _), v in vals.items():
        out.setdefault(name, {}).setdefault(grid, []).append(v)
    return out


def per_dispatch(d, counter, kernel_sub):
    grid = None
    if "@" in kernel_sub:
        kernel_sub, grid = kernel_sub.split("@", 1)
    if d.endswith(".json"):
        with open(d) as f:
            by_grid = json.load(f).get(kernel_sub, {})
        return [v for g, vs in by_grid.items() if grid is None or g == grid for v in vs]
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if base_name(name) != kernel_sub or row.get("Counter_Name") != counter:
                    continue
                if grid is not None and (row.get("Grid_Size") or row.get("Grid_Size_X")) != grid:
                    continue
                key = (path, row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(vals)))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    if sys.argv[1] == "--compact":
        json.dump(compact(sys.argv[2], sys.argv[3]), sys.stdout)
        print()
        return
    fetch_dir, write_dir = sys.argv[1], sys.argv[2]
    out = {}
    for spec in sys.argv[3:]:
        key, kernel = spec.split("=", 1) if "=" in spec else (spec, spec)
        f = per_dispatch(fetch_dir, "FETCH_SIZE", kernel)
        w = per_dispatch(write_dir, "WRITE_SIZE", kernel)
        e = {"kernel": kernel, "dispatches": [len(f), len(w)]}
        if f:
            e["fetch_bytes"] = 2 * 1024 * statistics.median(f)  # gfx950: FETCH_SIZE = half the bytes
        if w:
            e["write_bytes"] = 1024 * statistics.median(w)
        if f and w:
            e["bytes"] = e["fetch_bytes"] + e["write_bytes"]
        out[key] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

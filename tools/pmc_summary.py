"""Fold rocprofv3 --pmc counter CSVs per kernel: the median over dispatches
of every counter, for kernels whose base name starts with PREFIX.

    python tools/pmc_summary.py DIR [DIR ...] PREFIX > summary.json

Derived (per dispatch, then median), when the counters are present:
  lds_conflict_frac  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  lds_busy_frac      = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 XCDs * 32 CUs)
                       (LDS-array cycles per CU per GPU cycle)
  wait_inst_lds_frac = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  mfma_busy_frac     = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
"""
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic import base_name  # noqa: E402

CUS_PER_XCD = 32
XCDS = 8


def collect(dirs, prefix):
    per = {}  # (kernel, dir, dispatch) -> {counter: value}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = base_name(row.get("Kernel_Name") or row.get("Kernel-Name") or "")
                    if not name.startswith(prefix):
                        continue
                    disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                    key = (name, d, disp)
                    c = per.setdefault(key, {})
                    c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return per


def main():
    *dirs, prefix = sys.argv[1:]
    per = collect(dirs, prefix)
    by_kernel = {}
    for (name, d, _), c in per.items():
        by_kernel.setdefault(name, {}).setdefault(d, []).append(c)
    out = {}
    for name, runs in by_kernel.items():
        counters = {}
        derived = {}
        for d, lst in runs.items():
            for c in lst:
                for k, v in c.items():
                    counters.setdefault(k, []).append(v)
                g = c.get("GRBM_GUI_ACTIVE")
                if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
                    derived.setdefault("lds_conflict_frac", []).append(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"])
                if g and "SQ_LDS_IDX_ACTIVE" in c:
                    derived.setdefault("lds_busy_frac", []).append(
                        c["SQ_LDS_IDX_ACTIVE"] / (g / XCDS * XCDS * CUS_PER_XCD))
                if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_LDS" in c:
                    derived.setdefault("wait_inst_lds_frac", []).append(c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"])
                if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    derived.setdefault("mfma_busy_frac", []).append(
                        c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / XCDS * XCDS * CUS_PER_XCD * 4))
        out[name] = {"dispatches": max(len(v) for v in counters.values()),
                     "counters_median": {k: statistics.median(v) for k, v in sorted(counters.items())},
                     "derived_median": {k: round(statistics.median(v), 4) for k, v in sorted(derived.items())}}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

"""One-line summary of a bench.py JSON line's streaming extras (A/B runs)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("extra", {})


def g(*path):
    x = e
    for p in path:
        if not isinstance(x, dict) or p not in x:
            return None
        x = x[p]
    return x


print("quad", d["ms_per_step"], d["roofline"]["frac"],
      "| elided", g("rechunk_mean", "elided", "ms"), "materialised", g("rechunk_mean", "materialised", "ms"),
      "| share", g("rechunk_mean_share", "rows_6250", "ms"), g("rechunk_mean_share", "rows_7000", "ms"),
      "| config1", g("config1", "ms"), g("config1", "roofline", "frac"),
      "| vorticity", g("vorticity", "ms"), g("vorticity", "roofline", "frac"),
      "| checks_failed", d.get("checks_failed"))

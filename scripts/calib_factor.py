"""FETCH_SIZE factor of a workload's kernel from scripts/gpu_calib.sh passes:
known bytes of the spaced layout / its FETCH_SIZE, and the packed layout's
calibrated read bytes.  usage: python scripts/calib_factor.py DIR WORKLOAD KERNEL_SUBSTRING"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import mean, pick, read_counters  # noqa: E402

d, wl, kn = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
res = {}
for lay in ("packed", "spaced"):
    meta = json.loads((d / f"{wl}_{lay}.json").read_text().strip().splitlines()[-1])
    c = read_counters(d / f"{wl}_{lay}")
    k = pick(c, kn)
    vals = c[k]["FETCH_SIZE"][-meta["reps"]:]  # the timed kernel's last reps dispatches
    res[lay] = (meta, mean(vals) * 1024, k, len(c[k]["FETCH_SIZE"]))
meta_s, fetch_s, k, nd = res["spaced"]
factor = meta_s["known_read_bytes"] / fetch_s
fetch_p = res["packed"][1]
print(json.dumps({"workload": wl, "kernel": k, "spaced_known_read_bytes": meta_s["known_read_bytes"],
                  "spaced_fetch_size_bytes": round(fetch_s), "factor": round(factor, 4),
                  "packed_fetch_size_bytes": round(fetch_p),
                  "packed_read_bytes_calibrated": round(fetch_p * factor),
                  "dispatches": nd}))

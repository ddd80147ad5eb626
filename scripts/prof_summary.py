"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py next to the
bench line it produced: per-kernel stats, and the ICRC kernel's mean over the
timed launches only (the last `steps` dispatches) to compare with the bench's
HIP-event mean (kernel_ms_mean)."""
import csv
import json
import sys
from pathlib import Path

d, bench_json = Path(sys.argv[1]), Path(sys.argv[2])
needle = sys.argv[3] if len(sys.argv) > 3 else "::icrc_"
stats = next(d.rglob("*kernel_stats.csv"))
trace = next(d.rglob("*kernel_trace.csv"))
print(f"== {stats.name}")
print(stats.read_text().strip())
rows = [r for r in csv.DictReader(open(trace)) if needle in r["Kernel_Name"]]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
bench = json.loads(bench_json.read_text().strip().splitlines()[-1])
k = bench["steps"]
timed = durs[-k:]
print(f"== {needle} dispatches: {len(durs)} (warmup {len(durs) - k} + timed {k})")
print(f"rocprof mean over timed dispatches: {sum(timed) / len(timed):.4f} ms "
      f"(min {min(timed):.4f}, max {max(timed):.4f})")
print(f"bench HIP-event kernel_ms_mean:     {bench['kernel_ms_mean']:.4f} ms  "
      f"(profiled run is a separate process; the bench line is from its own run)")

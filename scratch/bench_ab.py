"""A/B of library builds through bench.py: for each round, each workload and
each ROCE_ICRC_LIB, one bench.py child process (no CPU baseline, no e2e);
prints value GiB/s and kernel ms.
usage: python scratch/bench_ab.py --workloads cfg2,cfg3 --rounds 3 lib1.so lib2.so ..."""
import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

ap = argparse.ArgumentParser()
ap.add_argument("--workloads", default="cfg2")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--bench-args", default="", help="extra bench.py arguments, e.g. '--lanes 16'")
ap.add_argument("libs", nargs="+")
args = ap.parse_args()
for rnd in range(args.rounds):
    for wl in args.workloads.split(","):
        for lib in args.libs:
            env = dict(os.environ, ROCE_ICRC_LIB=str(Path(lib).resolve()))
            r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--workload", wl,
                                "--no-cpu-baseline", "--no-e2e"] + args.bench_args.split(), env=env, timeout=300,
                               capture_output=True, text=True)
            # exit status 3: the line was printed but a check failed (diagnostic
            # builds that skip work do that); anything else is an error
            if r.returncode not in (0, 3):
                print(r.stderr[-2000:], flush=True)
                sys.exit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(f"r{rnd} {wl:5s} {Path(lib).name:12s} {d['value']:9.1f} GiB/s "
                  f"kernel {d['kernel_ms_mean']:.4f} ms frac {d['roofline']['frac']}"
                  + ("" if r.returncode == 0 else "  (CHECK FAILED)"), flush=True)

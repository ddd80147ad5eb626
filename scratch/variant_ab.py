"""A/B of kernel variants through bench.py, one child process per run.
A variant is LABEL=ENV1=V1,ENV2=V2@--bench --args (env and bench args both
optional), e.g.  g8v1=@--lanes 8   g4v2=ROCE_ICRC_CHUNKS=2@--lanes 4
usage: python scratch/variant_ab.py --workloads cfg2,cfg3 --rounds 3 [--warmup W --steps K] VARIANT..."""
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
ap.add_argument("--warmup", type=int, default=30)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("variants", nargs="+")
args = ap.parse_args()
vs = []
for v in args.variants:
    label, rest = v.split("=", 1)
    envs, _, extra = rest.partition("@")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    vs.append((label, env, extra.split()))
for rnd in range(args.rounds):
    for wl in args.workloads.split(","):
        for label, env, extra in vs:
            r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--workload", wl,
                                "--no-cpu-baseline", "--no-e2e", "--warmup", str(args.warmup),
                                "--steps", str(args.steps)] + extra,
                               env=dict(os.environ, **env), timeout=300, capture_output=True,
                               text=True)
            if r.returncode != 0:
                print(r.stderr[-3000:], flush=True)
                sys.exit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(f"r{rnd} {wl:5s} {label:10s} {d['value']:9.1f} GiB/s kernel "
                  f"{d['kernel_ms_mean']:.4f} ms frac {d['roofline']['frac']} "
                  f"{json.dumps(d.get('checks', {}))[:120]}", flush=True)

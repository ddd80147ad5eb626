"""Where the ~6 us between back-to-back launches comes from (bench.py's wall
time per step exceeds its HIP-event kernel time by that much): K launches of
the cfg2 / cfg5 kernels timed by wall clock with (a) two events around every
launch (bench.py's loop), (b) events around the whole run only, (c) no events,
(d) one event per launch (after it).  Prints wall us per step and, for (a), the
mean event-bracketed kernel time.

usage: python scratch/step_gap.py [--steps 100] [--reps 3]"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()

eng = IcrcEngine(0)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev)
sp = s.cuda_stream
K = args.steps


def run(step, mode):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(20):  # warm-up, back to back
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mode == "ends":
        e0.record(s)
    for a, b in evs:
        if mode == "each":
            a.record(s)
        step()
        if mode in ("each", "after"):
            b.record(s)
    if mode == "ends":
        e1.record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / K * 1e6
    extra = ""
    if mode == "each":
        extra = f" kernel {np.mean([a.elapsed_time(b) for a, b in evs]) * 1e3:.1f} us"
    if mode == "ends":
        extra = f" events {e0.elapsed_time(e1) / K * 1e3:.1f} us/step"
    return f"{mode:5s} wall {wall:.1f} us/step{extra}"


n = 1 << 20
buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
d = torch.from_numpy(buf).to(dev)
del buf
out = torch.zeros(n, dtype=torch.int32, device=dev)
step2 = lambda: eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)  # noqa: E731
for r in range(args.reps):
    for mode in ("each", "ends", "none", "after"):
        print("cfg2", r, run(step2, mode), flush=True)
del d, out
n = 1 << 24
buf, stride, flen = synth.uniform_frames(n, 64, seed=synth.SEED_CFG2)
d = torch.from_numpy(buf).to(dev)
del buf
out = torch.zeros(n, dtype=torch.int32, device=dev)
step5 = lambda: eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)  # noqa: E731
for r in range(args.reps):
    for mode in ("each", "ends", "none", "after"):
        print("cfg5", r, run(step5, mode), flush=True)

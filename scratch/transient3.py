"""Bisect why bench.py's first ICRC launches dip while transient2.py's do not
(same box).  Mode (argv[1]):
  probe     -- transient2.py's order: engine, data, 100 STREAM launches, 60 ICRC
  torchfirst-- torch.cuda.set_device(0) before the engine (bench.py's order)
  synced    -- two synchronised STREAM launches before the series (measure_ceiling)
  benchcls  -- bench.py's Strided workload object and measure_ceiling()
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
sys.path.insert(0, str(ROOT))
mode = sys.argv[1]
if mode in ("torchfirst", "benchcls"):
    torch.cuda.set_device(0)
from roce_icrc import IcrcEngine, synth  # noqa: E402

eng = IcrcEngine(0)
s = torch.cuda.current_stream()
sp = s.cuda_stream
n = 1 << 20


def series(fn, k):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(k)]
    for a, b in evs:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b) * 1e3) for a, b in evs]


if mode in ("benchcls", "benchcls_series"):
    import bench
    W = bench.Strided(torch, eng, torch.device("cuda", 0), 4096, n, 0x1C2C0001, 0, 1)
    if mode == "benchcls":
        _, _, pre = bench.measure_ceiling(torch, eng, W, s, sp, torch.device("cuda", 0))
        pre = [round(x * 1e6) for x in pre]
    else:
        sink = torch.zeros(4, dtype=torch.int32, device="cuda")
        nb = W.d_frames.numel() // 16 * 16
        pre = series(lambda: eng.stream_read_dev(W.d_frames, nb, sink, stream=sp), 100)

    def icrc():
        W.step(sp)
elif mode.startswith("mc"):  # measure_ceiling variants, probe data
    buf, stride, flen = synth.uniform_frames(n, 4096)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    dev = torch.device("cuda", 0)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    nb = d.numel() // 16 * 16

    def launch():
        eng.stream_read_dev(d, nb, sink, stream=sp)
    if not mode.startswith("mc_nosync"):
        launch()
        torch.cuda.synchronize(dev)
        launch()
        torch.cuda.synchronize(dev)
    k = 124
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(k)]
    for a, b in evs:
        a.record(s)
        launch()
        b.record(s)
    torch.cuda.synchronize(dev)
    pre = [a.elapsed_time(b) * 1e-3 for a, b in evs]
    if mode == "mc_del":
        del evs

    def icrc():
        eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)
elif mode == "probe_ceiling":
    import types

    import bench
    buf, stride, flen = synth.uniform_frames(n, 4096)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    W = types.SimpleNamespace(d_frames=d)
    _, _, pre = bench.measure_ceiling(torch, eng, W, s, sp, torch.device("cuda", 0))

    def icrc():
        eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)
else:
    buf, stride, flen = synth.uniform_frames(n, 4096)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    nb = d.numel() // 16 * 16
    torch.cuda.synchronize()

    def icrc():
        eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)

    def stream():
        eng.stream_read_dev(d, nb, sink, stream=sp)

    if mode == "synced":
        stream()
        torch.cuda.synchronize()
        stream()
        torch.cuda.synchronize()
    pre = series(stream, 100)
if "_gap" in mode:  # idle gap (ms) between the pre-phase and the ICRC series
    import time
    time.sleep(float(mode.split("_gap")[1]) * 1e-3)
ge = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
ge[0].record(s)
t = series(icrc, 60)
pre_us = [round(x * 1e6) if x < 1 else x for x in pre]
print(mode, "pre n", len(pre), "pre_times", pre_us[:8], "...", pre_us[-8:], flush=True)
print(mode, "pre n", len(pre), "times", t, flush=True)
print(mode, "mean[5:25]", int(np.mean(t[5:25])), "mean[30:]", int(np.mean(t[30:])), flush=True)

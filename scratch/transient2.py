"""Per-launch times (us) of the cfg2 ICRC kernel after different pre-phases,
in a FRESH process per scenario (argv[1]):
  cold      -- upload, then the ICRC series
  stream    -- upload, 100 back-to-back STREAM-read launches, then the series
  stream400 -- the same with 400 STREAM launches (~250 ms)
  icrc      -- upload, 100 untimed ICRC launches, then the series
  spin      -- upload, 200 ms of a register-only busy kernel, then the series
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "/root/repo/roce-sim_amd")
from roce_icrc import IcrcEngine, synth  # noqa: E402

mode = sys.argv[1]
eng = IcrcEngine(0)
n = 1 << 20
buf, stride, flen = synth.uniform_frames(n, 4096)
d = torch.from_numpy(buf).cuda()
out = torch.zeros(n, dtype=torch.int32, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
sp = s.cuda_stream
nb = d.numel() // 16 * 16
torch.cuda.synchronize()


def icrc():
    eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)


def stream():
    eng.stream_read_dev(d, nb, sink, stream=sp)


def series(fn, k):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(k)]
    for a, b in evs:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b) * 1e3) for a, b in evs]


pre = []
if mode == "stream":
    pre = series(stream, 100)
elif mode == "stream20":
    pre = series(stream, 20)
elif mode == "stream400":
    pre = series(stream, 400)
elif mode == "icrc":
    pre = series(icrc, 100)
elif mode == "spin":
    x = torch.randn(4096, 4096, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        for _ in range(10):
            x = torch.sin(x)
        torch.cuda.synchronize()
t = series(icrc, 60)
print(mode, "pre_mean", int(np.mean(pre)) if pre else None, "times", t, flush=True)
print(mode, "mean[5:25]", int(np.mean(t[5:25])), "mean[30:]", int(np.mean(t[30:])), flush=True)

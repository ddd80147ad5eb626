"""Per-launch kernel times of the cfg2 ICRC kernel from a cold start: the
power-management transient that the driver's short warm-up (--warmup 5) puts
into the timed region.  Prints every launch time (us) of each series."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "/root/repo/roce-sim_amd")
from roce_icrc import IcrcEngine, synth  # noqa: E402

eng = IcrcEngine(0)
n = 1 << 20
buf, stride, flen = synth.uniform_frames(n, 4096)
d = torch.from_numpy(buf).cuda()
out = torch.zeros(n, dtype=torch.int32, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
sp = s.cuda_stream
nb = d.numel() // 16 * 16


def series(fn, k):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(k)]
    for a, b in evs:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b) * 1e3) for a, b in evs]


icrc = lambda: eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)  # noqa: E731
stream = lambda: eng.stream_read_dev(d, nb, sink, stream=sp)  # noqa: E731
mode = sys.argv[1] if len(sys.argv) > 1 else "all"
for name, fn, sleep, k in [("icrc-cold", icrc, 0.0, 80), ("icrc-after2s", icrc, 2.0, 80),
                           ("stream-after2s", stream, 2.0, 80), ("icrc-after-stream", icrc, 0.0, 80),
                           ("icrc-after0.2s", icrc, 0.2, 80)]:
    time.sleep(sleep)
    t = series(fn, k)
    print(name, "times", t, flush=True)
    print(name, "mean[5:25]", int(np.mean(t[5:25])), "mean[30:]", int(np.mean(t[30:])), flush=True)

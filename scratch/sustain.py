import sys, time, json
import numpy as np, torch
sys.path.insert(0, "/root/repo/roce-sim_amd")
from roce_icrc import IcrcEngine, synth
eng = IcrcEngine(0)
n = 1 << 20
buf, stride, flen = synth.uniform_frames(n, 4096)
d = torch.from_numpy(buf).cuda(); out = torch.zeros(n, dtype=torch.int32, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream(); sp = s.cuda_stream
nb = d.numel() // 16 * 16
def series(fn, k):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for a, b in evs:
        a.record(s); fn(); b.record(s)
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b) * 1e3) for a, b in evs]
for name, fn in [("icrc", lambda: eng.compute_strided_dev(d, stride, flen, n, out, stream=sp)),
                 ("stream", lambda: eng.stream_read_dev(d, nb, sink, stream=sp)),
                 ("icrc", lambda: eng.compute_strided_dev(d, stride, flen, n, out, stream=sp))]:
    time.sleep(2.0)
    t = series(fn, 200)
    print(name, "first10", t[:10], "p50", int(np.median(t)), "last50_mean", int(np.mean(t[-50:])), "min", min(t), "max", max(t), flush=True)

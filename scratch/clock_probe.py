"""GFX clock per launch from the diagnostic build (-DRICRC_BLOCK_TIMES): each
workgroup of the strided kernel records s_memrealtime (100 MHz) and s_memtime
(shader clock) at start and end; cycles / real time = the clock it ran at.
Prints, per launch of a cold series: kernel us (HIP events), the median
workgroup duration and the median GFX clock in MHz.

Usage: ROCE_ICRC_LIB=scratch/libs/times.so python scratch/clock_probe.py [pre]
  pre = none | stream (100 STREAM-read launches first)
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402

pre = sys.argv[1] if len(sys.argv) > 1 else "none"
eng = IcrcEngine(0)
s = torch.cuda.current_stream()
sp = s.cuda_stream
nblk = torch.cuda.get_device_properties(0).multi_processor_count
n = 1 << 20
buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
d = torch.from_numpy(buf).cuda()
del buf
out = torch.zeros(n, dtype=torch.int32, device="cuda")
K = 60
slot = 32 * nblk
st = torch.zeros(K * slot, dtype=torch.uint8, device="cuda")
if pre == "stream":
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    nb = d.numel() // 16 * 16
    for _ in range(100):
        eng.stream_read_dev(d, nb, sink, stream=sp)
torch.cuda.synchronize()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
for i, (a, b) in enumerate(evs):
    a.record(s)
    eng.compute_strided_dev(d, stride, flen, n, out, st[i * slot:], stream=sp)
    b.record(s)
torch.cuda.synchronize()
raw = st.cpu().numpy()
rows = []
for i, (a, b) in enumerate(evs):
    t = raw[i * slot:(i + 1) * slot].view(np.uint64).reshape(2, nblk, 2).astype(np.int64)
    real = (t[0, :, 1] - t[0, :, 0]) * 10e-3  # us
    cyc = t[1, :, 1] - t[1, :, 0]
    mhz = cyc / real
    rows.append((round(a.elapsed_time(b) * 1e3), round(float(np.median(real))), round(float(np.median(mhz)))))
print(pre, "kernel_us", [r[0] for r in rows])
print(pre, "wg_med_us", [r[1] for r in rows])
print(pre, "gfx_MHz", [r[2] for r in rows], flush=True)

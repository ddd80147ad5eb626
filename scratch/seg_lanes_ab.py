"""Segmentation kernel A/B over lanes per packet (the access pattern: 64 / G
packets per wave in flight), bench's seg workload (2^20 x 4 KiB-PMTU SEND
packets from 256-KiB WRs), one event pair per series of launches, settings
interleaved round by round; the frames and words of every setting are compared
with the first setting's.  ROCE_ICRC_LIB selects the library build (round 6:
a variant with segment_kernel<5>, <6> instantiated and seg_log2g clamped at 6;
the shipped library stops at 16 lanes).

usage: python scratch/seg_lanes_ab.py [--lanes 8,16,32,64] [--rounds 3] [--launches 20]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
import torch  # noqa: E402
from roce_icrc import engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lanes", default="8,16,32,64")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--launches", type=int, default=20)
ap.add_argument("--pmtu", type=int, default=4096)
ap.add_argument("--msg", type=int, default=256 * 1024)
ap.add_argument("--pkts", type=int, default=1 << 20)
ap.add_argument("--tag", default="")
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng = E.IcrcEngine(0)
per = -(-a.msg // a.pmtu)
nwr = a.pkts // per
g = torch.Generator(device=dev)
g.manual_seed(6)
mr = torch.randint(0, 256, (nwr * a.msg,), dtype=torch.uint8, device=dev, generator=g)
rec = E.seg_wrs(nwr)
rec["op"] = E.SEG_SEND
rec["mr_offset"] = np.arange(nwr, dtype=np.uint64) * a.msg
rec["length"] = a.msg
rec["psn"] = (np.arange(nwr, dtype=np.uint64) * per) % (1 << 24)
rec["dqpn"] = 0x11
rec["flags"] = E.SEG_SIGNALED
npk, slot = E.segment_plan(rec, a.pmtu)
d_wrs = torch.from_numpy(rec.view(np.uint8)).to(dev)
frames = torch.empty(npk * slot, dtype=torch.uint8, device=dev)
lens = torch.empty(npk, dtype=torch.int32, device=dev)
icrc = torch.empty(npk, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
lanes = [int(x) for x in a.lanes.split(",")]


def launch():
    eng.segment_dev(mr, mr.numel(), d_wrs, nwr, a.pmtu, npk, frames, slot, lens, icrc,
                    stream=s.cuda_stream)


ref = None
flen_sum = None
for L in lanes:
    eng.set_lanes(L)
    frames.zero_()
    launch()
    torch.cuda.synchronize()
    if ref is None:
        ref = (frames.clone(), icrc.clone(), lens.clone())
        flen_sum = int(lens.to(torch.int64).sum())
    else:
        # both runs start from zeroed slots; bytes past a frame are zeros either way
        fa, fb = frames, ref[0]
        print(json.dumps({"lanes": L, "frames_equal": bool(torch.equal(fa, fb)),
                          "icrc_equal": bool(torch.equal(icrc, ref[1])),
                          "lens_equal": bool(torch.equal(lens, ref[2]))}), flush=True)
alg = nwr * a.msg + flen_sum + 8 * npk
res = {L: [] for L in lanes}
for r in range(a.rounds):
    for L in lanes:
        eng.set_lanes(L)
        for _ in range(5):
            launch()
        x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        x.record(s)
        for _ in range(a.launches):
            launch()
        y.record(s)
        y.synchronize()
        ms = x.elapsed_time(y) / a.launches
        res[L].append(ms)
        print(json.dumps({"tag": a.tag, "round": r, "lanes": L, "ms": round(ms, 4),
                          "frac": round(alg / ms / 1e6 / 8000, 4)}), flush=True)
nb = (nwr * a.msg) // 16 * 16
for _ in range(3):
    eng.stream_copy_dev(mr, frames, nb)
x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
x.record(s)
for _ in range(10):
    eng.stream_copy_dev(mr, frames, nb)
y.record(s)
y.synchronize()
ms = x.elapsed_time(y) / 10
print(json.dumps({"tag": a.tag, "summary": {L: [round(v, 4) for v in res[L]] for L in lanes},
                  "stream_copy_GBps": round(2 * nb / ms / 1e6, 1)}), flush=True)

"""Segmentation kernel exploration: lanes x MR alignment shift, GB/s of
algorithmic bytes (MR read + frames written).  ROCE_ICRC_LIB selects the
library build (e.g. the RICRC_ABLATE_FOLD diagnostic build)."""
import argparse, json, sys, time
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
import torch
from roce_icrc import engine as E

ap = argparse.ArgumentParser()
ap.add_argument("--lanes", default="8,16")
ap.add_argument("--shift", default="0,8")
ap.add_argument("--pmtu", type=int, default=4096)
ap.add_argument("--msg", type=int, default=256 * 1024)
ap.add_argument("--pkts", type=int, default=1 << 20)
ap.add_argument("--tag", default="")
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng = E.IcrcEngine(0)
per = -(-a.msg // a.pmtu)
nwr = a.pkts // per
mr = torch.randint(0, 256, (nwr * a.msg + 64,), dtype=torch.uint8, device=dev)
for shift in [int(x) for x in a.shift.split(",")]:
    rec = E.seg_wrs(nwr)
    rec["op"] = 0
    rec["mr_offset"] = np.arange(nwr, dtype=np.uint64) * a.msg + shift
    rec["length"] = a.msg
    rec["dqpn"] = 0x11
    npk, slot = E.segment_plan(rec, a.pmtu)
    d_wrs = torch.from_numpy(rec.view(np.uint8)).to(dev)
    frames = torch.empty(npk * slot, dtype=torch.uint8, device=dev)
    lens = torch.empty(npk, dtype=torch.int32, device=dev)
    icrc = torch.empty(npk, dtype=torch.int32, device=dev)
    flen_sum = None
    for lanes in [int(x) for x in a.lanes.split(",")]:
        eng.set_lanes(lanes)
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(15):
            eng.segment_dev(mr, mr.numel(), d_wrs, nwr, a.pmtu, npk, frames, slot, lens, icrc, stream=s)
        torch.cuda.synchronize()
        if flen_sum is None:
            flen_sum = int(lens.to(torch.int64).sum())
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for x, y in ev:
            x.record(); eng.segment_dev(mr, mr.numel(), d_wrs, nwr, a.pmtu, npk, frames, slot, lens, icrc, stream=s); y.record()
        torch.cuda.synchronize()
        ms = float(np.median([x.elapsed_time(y) for x, y in ev]))
        alg = nwr * a.msg + flen_sum + 8 * npk
        print(json.dumps({"tag": a.tag, "pmtu": a.pmtu, "shift": shift, "lanes": lanes, "ms": round(ms, 4),
                          "GBps_alg": round(alg / ms / 1e6, 1)}), flush=True)
nb = (nwr * a.msg) // 16 * 16
for _ in range(3):
    eng.stream_copy_dev(mr, frames, nb)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
for x, y in ev:
    x.record(); eng.stream_copy_dev(mr, frames, nb); y.record()
torch.cuda.synchronize()
ms = float(np.median([x.elapsed_time(y) for x, y in ev]))
dd = torch.empty_like(mr[:nb])
for _ in range(3):
    dd.copy_(mr[:nb])
torch.cuda.synchronize()
x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
x.record(); dd.copy_(mr[:nb]); y.record(); torch.cuda.synchronize()
print(json.dumps({"tag": a.tag, "stream_copy_GBps": round(2 * nb / ms / 1e6, 1),
                  "torch_copy_GBps": round(2 * nb / x.elapsed_time(y) / 1e6, 1)}), flush=True)

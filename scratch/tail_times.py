"""Per-workgroup start / end times of the bench workloads' kernels (diagnostic
library of scratch/diag_build.py, loaded through ROCE_ICRC_LIB): how long the
launch runs after its median workgroup is done (the tail) and how spread the
starts are.  Launches with a status buffer (the timer writes after its n
bytes), 30 back to back; the last one is read.

usage: ROCE_ICRC_LIB=scratch/libs/diag.so python scratch/tail_times.py"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402
from roce_icrc import engine as E  # noqa: E402

eng = IcrcEngine(0)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev)
sp = s.cuda_stream
NBLK = torch.cuda.get_device_properties(0).multi_processor_count


def report(tag, st, n, reps):
    off = (n + 15) & ~15
    t = st[off: off + 16 * NBLK].view(np.uint64).reshape(NBLK, 2).astype(np.int64)
    ok = t[:, 1] > 0
    t = t[ok]
    t0 = t[:, 0].min()
    start, end = (t[:, 0] - t0) * 1e-2, (t[:, 1] - t0) * 1e-2  # 100 MHz -> us
    print(json.dumps({
        "kernel": tag, "blocks": int(ok.sum()), "launch_us": round(float(end.max()), 2),
        "start_spread_us": round(float(start.max()), 2),
        "end_min_us": round(float(end.min()), 2), "end_med_us": round(float(np.median(end)), 2),
        "end_p90_us": round(float(np.percentile(end, 90)), 2), "end_max_us": round(float(end.max()), 2),
        "tail_us": round(float(end.max() - np.median(end)), 2),
        "xcd_end_med_us": [round(float(np.median(end[x::8])), 1) for x in range(8)],
        "xcd_start_med_us": [round(float(np.median(start[x::8])), 1) for x in range(8)]}), flush=True)


def run(tag, n, step, st, reps=30):
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    for r in range(3):
        step()
        torch.cuda.synchronize()
        report(f"{tag} #{r}", st.cpu().numpy(), n, reps)


def status(n):
    return torch.zeros(((n + 15) & ~15) + 16 * NBLK, dtype=torch.uint8, device=dev)


# cfg2: strided 4 KiB
n = 1 << 20
buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
d = torch.from_numpy(buf).to(dev)
del buf
out = torch.zeros(n, dtype=torch.int32, device=dev)
st = status(n)
run("cfg2 strided", n, lambda: eng.compute_strided_dev(d, stride, flen, n, out, st, stream=sp), st)
del d
# cfg5: 108-B strided
n = 1 << 24
buf, stride, flen = synth.uniform_frames(n, 64, seed=synth.SEED_CFG2)
d = torch.from_numpy(buf).to(dev)
del buf
out = torch.zeros(n, dtype=torch.int32, device=dev)
st = status(n)
run("cfg5 small", n, lambda: eng.compute_strided_dev(d, stride, flen, n, out, st, stream=sp), st)
del d, out, st
# cfg3: mixed MTU, verify (sorted)
n = 1 << 20
buf, offs, lens = synth.mixed_mtu_frames(n)
d = torch.from_numpy(buf).to(dev)
do = torch.from_numpy(offs.view(np.int64)).to(dev)
dl = torch.from_numpy(lens.view(np.int32)).to(dev)
del buf
ok = torch.zeros(n, dtype=torch.uint8, device=dev)
st = status(n)
eng.set_ragged_variant(E.RAGGED_SORTED)
run("cfg3 sorted verify", n, lambda: eng.verify_batch_dev(d, do, dl, n, ok, None, st, stream=sp), st)
del d, do, dl
# ack: 48-B frames packed, compute (compact)
n = 1 << 24
buf, offs, lens = synth.mixed_mtu_frames(n, mtus=(4,), opcode=0x11)
d = torch.from_numpy(buf).to(dev)
do = torch.from_numpy(offs.view(np.int64)).to(dev)
dl = torch.from_numpy(lens.view(np.int32)).to(dev)
del buf
out = torch.zeros(n, dtype=torch.int32, device=dev)
st = status(n)
eng.set_ragged_variant(E.RAGGED_COMPACT)
run("ack compact", n, lambda: eng.compute_batch_dev(d, do, dl, n, out, st, stream=sp), st)

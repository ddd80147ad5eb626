"""Per-wave clocks and claim counts of the sorted kernel's tail pool on cfg3
(diagnostic library: /tmp/pooldiag.diff over the round-6 pool source, loaded
through ROCE_ICRC_LIB): entry, sort done, window sets done, pool start, end
(100-MHz stamps, us from the launch's first entry), and per wave the pool sets
taken from its own workgroup, stolen from others, and probes.

usage: ROCE_ICRC_LIB=scratch/libs/pooldiag.so python scratch/pool_times.py"""
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
sp = torch.cuda.current_stream(dev).cuda_stream
NBLK = torch.cuda.get_device_properties(0).multi_processor_count
n = 1 << 20
buf, offs, lens = synth.mixed_mtu_frames(n)
d = torch.from_numpy(buf).to(dev)
do = torch.from_numpy(offs.view(np.int64)).to(dev)
dl = torch.from_numpy(lens.view(np.int32)).to(dev)
ok = torch.zeros(n, dtype=torch.uint8, device=dev)
off = (n + 15) & ~15
st = torch.zeros(off + 64 * 16 * NBLK, dtype=torch.uint8, device=dev)
eng.set_ragged_variant(E.RAGGED_SORTED)
for _ in range(30):
    eng.verify_batch_dev(d, do, dl, n, ok, None, st, stream=sp)
torch.cuda.synchronize()


def q(v):
    return {"min": round(float(v.min()), 1), "med": round(float(np.median(v)), 1), "max": round(float(v.max()), 1)}


for rep in range(3):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    eng.verify_batch_dev(d, do, dl, n, ok, None, st, stream=sp)
    ev[1].record()
    torch.cuda.synchronize()
    t = st.cpu().numpy()[off:].view(np.uint64).reshape(NBLK, 16, 8).astype(np.int64)
    t0 = t[:, :, 0].min()
    us = (t[:, :, :5] - t0) * 1e-2
    blk_end = us[:, :, 4].max(1)
    res = {"rep": rep, "kernel_ms": round(ev[0].elapsed_time(ev[1]), 4),
           "entry": q(us[:, :, 0]), "sorted": q(us[:, :, 1]), "sets_done": q(us[:, :, 2]),
           "pool_start": q(us[:, :, 3]), "end": q(us[:, :, 4]), "block_end": q(blk_end),
           "own_sets": int(t[:, :, 5].sum()), "stolen_sets": int(t[:, :, 6].sum()),
           "probes": int(t[:, :, 7].sum()), "probes_per_wave_max": int(t[:, :, 7].max()),
           "pool_time_per_wave_med_us": round(float(np.median(us[:, :, 4] - us[:, :, 3])), 1)}
    print(json.dumps(res), flush=True)

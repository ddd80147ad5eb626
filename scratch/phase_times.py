"""Per-wave phase clocks of the sorted ragged kernel on cfg3 (diagnostic
library built with -DRICRC_PHASE_TIMES, loaded through ROCE_ICRC_LIB): for
the first window of every workgroup, 100-MHz stamps at kernel entry (T0),
tables staged (T1), keys counted (T2, per wave), after the count barrier (T3),
sort done (T4), the wave's last set done (T5), the window's barrier (T6) and
the end (T7).  Prints medians and spreads in microseconds from the launch's
first T0.

usage: ROCE_ICRC_LIB=scratch/libs/phase.so python scratch/phase_times.py"""
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
ends = []
for rep in range(6):
    eng.verify_batch_dev(d, do, dl, n, ok, None, st, stream=sp)
    torch.cuda.synchronize()
    t = st.cpu().numpy()[off:].view(np.uint64).reshape(NBLK, 16, 8).astype(np.int64)
    t0 = t[:, :, 0].min()
    us = (t - t0) * 1e-2
    res = {"rep": rep}
    for k, name in enumerate(["entry", "tables", "keys", "count_bar", "sorted", "sets_done", "win_bar", "end"]):
        v = us[:, :, k]
        res[name] = {"min": round(float(v.min()), 2), "med": round(float(np.median(v)), 2),
                     "max": round(float(v.max()), 2)}
    blk = us[:, 0, :]
    res["per_block_phase_med_us"] = {
        "tables": round(float(np.median(blk[:, 1] - blk[:, 0])), 2),
        "keys": round(float(np.median(us[:, :, 2].max(1) - blk[:, 1])), 2),
        "scan_scatter": round(float(np.median(blk[:, 4] - blk[:, 3])), 2),
        "sets": round(float(np.median(blk[:, 6] - blk[:, 4])), 2),
        "wave_set_end_spread": round(float(np.median(us[:, :, 5].max(1) - us[:, :, 5].min(1))), 2)}
    ends.append(us[:, :, 6].max(1) - us[:, :, 0].min(1))  # per block: window barrier - entry
    print(json.dumps(res), flush=True)
E_ = np.array(ends)  # reps x blocks: each block's own duration
c = np.corrcoef(E_[1:])
print(json.dumps({"block_duration_corr_between_reps": [[round(float(x), 2) for x in r] for r in c],
                  "xcd_mean_duration_us": [[round(float(E_[r, x::8].mean()), 1) for x in range(8)] for r in range(1, 6)],
                  "within_xcd_std_us": [round(float(np.mean([E_[r, x::8].std() for x in range(8)])), 2) for r in range(1, 6)],
                  "block_duration_std_us": [round(float(E_[r].std()), 2) for r in range(1, 6)]}), flush=True)

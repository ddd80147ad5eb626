"""Per-workgroup start / end clocks of the compact (ACK) kernel on 2^24 packed
48-B ACK frames (diagnostic library: thread 0 of each workgroup writes two
100-MHz stamps after the batch's words, loaded through ROCE_ICRC_LIB).
usage: ROCE_ICRC_LIB=scratch/libs/ackt.so python scratch/ack_times.py"""
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
n = 1 << 24
buf, offs, lens = synth.mixed_mtu_frames(n, mtus=(4,), opcode=0x11, seed=0x1C2C0007)
d = torch.from_numpy(buf).to(dev)
do = torch.from_numpy(offs.view(np.int64)).to(dev)
dl = torch.from_numpy(lens.view(np.int32)).to(dev)
nw = ((n + 3) & ~3) + 4 * NBLK
out = torch.zeros(nw, dtype=torch.int32, device=dev)
eng.set_ragged_variant(E.RAGGED_COMPACT)
for _ in range(30):
    eng.compute_batch_dev(d, do, dl, n, out, stream=sp)
torch.cuda.synchronize()
for rep in range(4):
    eng.compute_batch_dev(d, do, dl, n, out, stream=sp)
    torch.cuda.synchronize()
    t = out.cpu().numpy()[(n + 3) & ~3:].view(np.uint64).reshape(NBLK, 2).astype(np.int64)
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) * 1e-2, (t[:, 1] - t0) * 1e-2
    dur = en - st
    print(json.dumps({"rep": rep, "launch_us": round(float(en.max()), 1),
                      "start_spread": round(float(st.max()), 1),
                      "end_min_med_max": [round(float(x), 1) for x in (en.min(), np.median(en), en.max())],
                      "dur_mean_std": [round(float(dur.mean()), 1), round(float(dur.std()), 2)],
                      "tail_after_mean_end": round(float(en.max() - en.mean()), 1),
                      "xcd_end_med": [round(float(np.median(en[x::8])), 1) for x in range(8)],
                      "xcd_start_med": [round(float(np.median(st[x::8])), 1) for x in range(8)]}), flush=True)

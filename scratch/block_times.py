"""Per-workgroup start/end clocks of the lane-group kernels (diagnostic build
with -DRICRC_BLOCK_TIMES, loaded through ROCE_ICRC_LIB): how long the last
workgroup runs after the first one is done (the launch tail).

Usage: ROCE_ICRC_LIB=scratch/libs/times.so python scratch/block_times.py
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402


def report(tag, st, nblk):
    t = st[: 16 * nblk].view(np.uint64).reshape(nblk, 2).astype(np.int64)
    t0 = t[:, 0].min()
    start, end = (t[:, 0] - t0) * 10e-3, (t[:, 1] - t0) * 10e-3  # 100 MHz -> us
    dur = end - start
    print(json.dumps({"kernel": tag, "blocks": nblk, "start_spread_us": float(start.max()),
                      "end_min_us": float(end.min()), "end_med_us": float(np.median(end)),
                      "end_max_us": float(end.max()), "dur_min_us": float(dur.min()),
                      "dur_max_us": float(dur.max()),
                      "tail_frac": float((end.max() - np.median(end)) / end.max()),
                      # workgroup b runs on XCD b % 8 (round-robin dispatch)
                      "xcd_end_med_us": [round(float(np.median(end[x::8])), 1) for x in range(8)],
                      "xcd_start_med_us": [round(float(np.median(start[x::8])), 1)
                                           for x in range(8)]}), flush=True)


def main():
    eng = IcrcEngine(0)
    s = torch.cuda.current_stream()
    nblk = torch.cuda.get_device_properties(0).multi_processor_count
    n = 1 << 20
    buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
    d = torch.from_numpy(buf).cuda()
    del buf
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for r in range(40):
        eng.compute_strided_dev(d, stride, flen, n, out, st, stream=s.cuda_stream)
        if r >= 36:
            s.synchronize()
            report("strided cfg2", st.cpu().numpy(), nblk)
    del d
    buf, offs, lens = synth.mixed_mtu_frames(n)
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    for r in range(40):
        eng.compute_batch_dev(d, do, dl, n, out, st, stream=s.cuda_stream)
        if r >= 36:
            s.synchronize()
            report("ragged cfg3", st.cpu().numpy(), nblk)


if __name__ == "__main__":
    main()

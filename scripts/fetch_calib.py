"""FETCH_SIZE calibration on a kernel's OWN access pattern (MI355X_MICROARCH
section HBM: widths other than 16-B/lane streaming reads are uncalibrated).

Runs one bench workload's ICRC kernel over one of two layouts of the same
frames:
  packed  -- the bench layout (cfg3: back to back; cfg2 / cfg5: stride = len),
  spaced  -- every frame at a 128-byte-aligned start, frames padded to whole
             128-B lines, so no HBM line is shared by two frames and every
             line the kernel touches is read exactly once: the HBM bytes the
             kernel must fetch are KNOWN (lines x 128 + descriptors).
Under `rocprofv3 --pmc FETCH_SIZE` the spaced run gives the factor
known bytes / FETCH_SIZE for this kernel's load pattern (G = 4 / G = 8 group
runs of 64 / 128 B for cfg3, lane-per-packet batches for cfg5, ...); the
packed run's FETCH_SIZE times that factor is the workload's HBM read traffic.

usage (on the GPU box, one process per pass):
  rocprofv3 --pmc FETCH_SIZE -d DIR -o run -- python3 scripts/fetch_calib.py \
      --workload cfg3 --layout spaced
prints one JSON line: the layout, packets, the known bytes of the spaced run.
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402

LINE = 128


def spaced(buf, offs, lens):
    """The same frames, each at a 128-B-aligned start in whole lines."""
    slots = ((lens.astype(np.uint64) + LINE - 1) // LINE) * LINE
    noffs = np.zeros_like(offs)
    if offs.size > 1:
        noffs[1:] = np.cumsum(slots[:-1])
    out = np.zeros(int(slots.sum()), np.uint8)
    for s in range(0, offs.size, 1 << 16):
        e = min(offs.size, s + (1 << 16))
        for i in range(s, e):
            o, n, l = int(noffs[i]), int(offs[i]), int(lens[i])
            out[o:o + l] = buf[n:n + l]
    return out, noffs, int(slots.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3", choices=("cfg2", "cfg3", "cfg5"))
    ap.add_argument("--layout", default="packed", choices=("packed", "spaced"))
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--time", type=int, default=0, help="also time this many launches")
    a = ap.parse_args()
    eng = IcrcEngine(0)
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    if a.workload == "cfg3":
        n = a.packets or 1 << 20
        buf, offs, lens = synth.mixed_mtu_frames(n, seed=synth.SEED_CFG3)
    else:
        n = a.packets or (1 << 20 if a.workload == "cfg2" else 1 << 24)
        pay = 4096 if a.workload == "cfg2" else 64
        buf, stride, flen = synth.uniform_frames(n, pay, seed=synth.SEED_CFG2)
        offs = np.arange(n, dtype=np.uint64) * stride
        lens = np.full(n, flen, np.uint32)
    if a.layout == "spaced":
        if a.workload == "cfg3":
            buf, offs, line_bytes = spaced(buf, offs, lens)
        else:  # strided: stride rounded up to whole lines (the kernel reads its batches whole)
            flen = int(lens[0])
            s2 = (flen + LINE - 1) // LINE * LINE
            b2 = np.zeros(n * s2, np.uint8)
            b2.reshape(n, s2)[:, :flen] = buf.reshape(n, flen)
            buf, offs, line_bytes = b2, np.arange(n, dtype=np.uint64) * s2, n * s2
    else:
        line_bytes = None
    d = torch.from_numpy(buf).to(dev)
    del buf
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    if a.workload == "cfg3":
        d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_l = torch.from_numpy(lens.view(np.int32)).to(dev)
        ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        # trailers filled by the compute path, then the timed kernel: verify (as bench)
        eng.compute_batch_dev(d, d_o, d_l, n, out, stream=sp)
        tr = (d_o + d_l.to(torch.int64) - 4)
        idx = tr[:, None] + torch.arange(4, device=dev)[None, :]
        d[idx.reshape(-1)] = out.view(torch.uint8).reshape(-1)
        torch.cuda.synchronize()

        def step():
            eng.verify_batch_dev(d, d_o, d_l, n, ok, stream=sp)
        desc_bytes = 12 * n  # offsets (8 B) + lengths (4 B) read once
        out_bytes = n  # verdicts written
    else:
        stride = int(offs[1] - offs[0]) if n > 1 else int(lens[0])

        def step():
            eng.compute_strided_dev(d, stride, int(lens[0]), n, out, stream=sp)
        desc_bytes = 0
        out_bytes = 4 * n
    for _ in range(a.reps):
        step()
    torch.cuda.synchronize()
    ms = None
    if a.time:  # (not under the profiler) HIP-event median over `time` launches
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.time)]
        for e0, e1 in ev:
            e0.record()
            step()
            e1.record()
        torch.cuda.synchronize()
        ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
    print(json.dumps({"workload": a.workload, "layout": a.layout, "packets": n, "reps": a.reps,
                      "kernel_ms_median": ms,
                      "frame_line_bytes": line_bytes, "descriptor_bytes": desc_bytes,
                      "known_read_bytes": None if line_bytes is None else line_bytes + desc_bytes,
                      "output_bytes": out_bytes}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Batch launches beside other contexts' resident per-packet service waves.

The reference calls compute_icrc from a 10-thread gRPC pool
(src/sanity_side.py:383); through ricrc_icrc every such thread owns a
library context whose service wave holds one CU's LDS while it runs.  This
times compute_strided_dev on context A (cfg2-shaped 4 KiB frames) with K of
those threads calling ricrc_icrc back to back the whole time, K = 0, 1, 4,
10, and checks every batch word and every per-packet answer.

usage: python scripts/svc_contention.py [--packets N] [--reps R] [--ks 0,1,4,10]
prints one JSON line: kernel ms (median, p90) per K and the slowdown vs K = 0.
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "roce-sim_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]


def run(packets: int = 1 << 18, reps: int = 40, ks=(0, 1, 4, 10)) -> dict:
    import torch

    import icrc_oracle as o  # checker only
    from conftest import oracle_batch
    from roce_icrc import IcrcEngine, synth
    from roce_icrc import engine as E

    buf, stride, flen = synth.uniform_frames(packets, 4096, seed=0x5EC)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=packets)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(packets, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    eng = IcrcEngine(0)
    frame = o.sim_send_success_frame()
    res = {"packets": packets, "frame_bytes": flen, "reps": reps, "per_k": {}}
    base = None
    for k in ks:
        stop = threading.Event()
        counts, errors = [0] * k, []

        def caller(t):
            try:
                while not stop.is_set():
                    if E.icrc(frame)[0] != 0x1BE21D75:
                        errors.append(t)
                        return
                    counts[t] += 1
            except Exception as ex:  # noqa: BLE001 (reported)
                errors.append(repr(ex))

        th = [threading.Thread(target=caller, args=(t,), daemon=True) for t in range(k)]
        for x in th:
            x.start()
        time.sleep(0.05)  # every thread's wave is resident
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(reps)]
        c0 = sum(counts)
        t0 = time.perf_counter()
        for a, b in evs:
            a.record(s)
            eng.compute_strided_dev(d, stride, flen, packets, out, stream=s.cuda_stream)
            b.record(s)
        s.synchronize()
        wall = time.perf_counter() - t0
        c1 = sum(counts)
        stop.set()
        for x in th:
            x.join(timeout=30)
        ms = np.array([a.elapsed_time(b) for a, b in evs])
        ok = bool((out.cpu().numpy().view(np.uint32) == want).all())
        med = float(np.median(ms))
        base = base or med
        res["per_k"][str(k)] = {
            "kernel_ms_median": round(med, 4), "kernel_ms_p90": round(float(np.percentile(ms, 90)), 4),
            "kernel_ms_max": round(float(ms.max()), 4), "slowdown": round(med / base, 4),
            "batch_bit_exact": ok, "icrc_calls_during_batches": c1 - c0,
            "icrc_calls_per_s_during": round((c1 - c0) / wall, 1), "errors": errors[:3]}
        out.zero_()
    eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--ks", default="0,1,4,10")
    a = ap.parse_args()
    print(json.dumps(run(a.packets, a.reps, tuple(int(x) for x in a.ks.split(",")))), flush=True)


if __name__ == "__main__":
    main()

"""Kernel exploration on one GPU: time the ICRC kernel for every lanes-per-packet
choice on the BASELINE configs, next to the STREAM-style read ceiling.

Usage: python scripts/explore.py [--cfg 2,3,5] [--reps 10]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402


def timed(fn, reps, stream):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    stream.synchronize()
    ts = []
    for _ in range(reps):
        ev[0].record(stream)
        fn()
        ev[1].record(stream)
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e-3)
    return float(np.median(ts)), float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="2,5,3")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lanes", default="1,2,4,8,16,32,64")
    args = ap.parse_args()
    eng = IcrcEngine(0)
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    lanes = [int(x) for x in args.lanes.split(",")]
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    for cfg in args.cfg.split(","):
        t0 = time.time()
        if cfg in ("2", "5"):
            n = 1 << 20 if cfg == "2" else 1 << 24
            pay = 4096 if cfg == "2" else 64
            buf, stride, flen = synth.uniform_frames(n, pay, seed=synth.SEED_CFG2)
            cov = (flen - 4) * n
            d = torch.from_numpy(buf).cuda()
            del buf
            out = torch.zeros(n, dtype=torch.int32, device="cuda")
            nbytes = d.numel() // 16 * 16
            med, mn = timed(lambda: eng.stream_read_dev(d, nbytes, sink, stream=sp), args.reps, s)
            print(json.dumps({"cfg": cfg, "kernel": "stream_read", "bytes": nbytes,
                              "GBps_med": nbytes / med / 1e9, "GBps_best": nbytes / mn / 1e9}),
                  flush=True)
            for g in lanes:
                eng.set_lanes(g)
                med, mn = timed(lambda: eng.compute_strided_dev(d, stride, flen, n, out, stream=sp),
                                args.reps, s)
                print(json.dumps({"cfg": cfg, "lanes": g, "ms": med * 1e3,
                                  "GiBps": cov / med / 2**30, "GBps_alg": (cov + 4 * n) / med / 1e9,
                                  "GiBps_best": cov / mn / 2**30}), flush=True)
            eng.set_lanes(0)
            del d, out
        elif cfg == "3":
            n = 1 << 20
            buf, offs, lens = synth.mixed_mtu_frames(n)
            cov = synth.covered_bytes(lens)
            d = torch.from_numpy(buf).cuda()
            do = torch.from_numpy(offs.view(np.int64)).cuda()
            dl = torch.from_numpy(lens.view(np.int32)).cuda()
            out = torch.zeros(n, dtype=torch.int32, device="cuda")
            ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
            for g in lanes:
                eng.set_lanes(g)
                med, mn = timed(lambda: eng.compute_batch_dev(d, do, dl, n, out, stream=sp),
                                args.reps, s)
                print(json.dumps({"cfg": cfg, "mode": "compute", "lanes": g, "ms": med * 1e3,
                                  "GiBps": cov / med / 2**30}), flush=True)
                med, mn = timed(lambda: eng.verify_batch_dev(d, do, dl, n, ok, stream=sp),
                                args.reps, s)
                print(json.dumps({"cfg": cfg, "mode": "verify", "lanes": g, "ms": med * 1e3,
                                  "GiBps": cov / med / 2**30}), flush=True)
            eng.set_lanes(0)
            del d, do, dl, out, ok
        elif cfg.startswith("u"):
            # homogeneous frames of payload P ("u256"): the strided kernel and the
            # ragged kernel (offsets i * stride) on the same buffer, per lane setting
            pay = int(cfg[1:])
            flen0 = pay + 44
            n = min(1 << 24, (2 << 30) // flen0)
            buf, stride, flen = synth.uniform_frames(n, pay, seed=synth.SEED_CFG2)
            cov = (flen - 4) * n
            d = torch.from_numpy(buf).cuda()
            del buf
            do = torch.arange(n, dtype=torch.int64, device="cuda") * stride
            dl = torch.full((n,), flen, dtype=torch.int32, device="cuda")
            out = torch.zeros(n, dtype=torch.int32, device="cuda")
            for g in lanes:
                eng.set_lanes(g)
                med, _ = timed(lambda: eng.compute_strided_dev(d, stride, flen, n, out, stream=sp),
                               args.reps, s)
                med2, _ = timed(lambda: eng.compute_batch_dev(d, do, dl, n, out, stream=sp),
                                args.reps, s)
                print(json.dumps({"cfg": cfg, "lanes": g, "n": n, "strided_GiBps": cov / med / 2**30,
                                  "ragged_GiBps": cov / med2 / 2**30}), flush=True)
            eng.set_lanes(0)
            del d, do, dl, out
        print(json.dumps({"cfg": cfg, "wall_s": time.time() - t0}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

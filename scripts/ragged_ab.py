#!/usr/bin/env python3
"""A/B of library builds (ROCE_ICRC_LIB) on device-resident ragged batches:
the responder's tiny frames (ACK 48 B, atomic ack 56 B, 104 B, a packed mix
of 44-128 B) and cfg3's mixed MTU, compute and verify.  Kernel time is the
median of R launches between HIP events on the launch stream; every answer is
checked against the C oracle (checker only).

usage: python scripts/ragged_ab.py [--rounds 2] [--cases u4,u12,u60,mix,cfg3] lib1.so [lib2.so ...]
prints one JSON line per (round, lib, case, mode); one child process per
(round, lib), rounds interleaved.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def make_case(name: str):
    import numpy as np
    from roce_icrc import synth
    if name == "cfg3":
        return synth.mixed_mtu_frames(1 << 20)
    if name == "mix":  # packed, dword-aligned frames of 44..128 B
        return synth.mixed_mtu_frames(1 << 22, mtus=tuple(range(0, 88, 4)), seed=12)
    pay = int(name[1:])
    n = 1 << 24 if pay <= 12 else 1 << 22
    buf, stride, flen = synth.uniform_frames(n, pay, seed=synth.SEED_CFG5)
    return buf, np.arange(n, dtype=np.uint64) * np.uint64(stride), np.full(n, flen, np.uint32)


def child(cases: list[str], reps: int) -> None:
    sys.path[:0] = [str(ROOT / "roce-sim_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
    import numpy as np
    import torch
    from conftest import oracle_batch  # checker only
    from roce_icrc import IcrcEngine, synth

    eng = IcrcEngine(0)
    s = torch.cuda.current_stream()
    lib = os.environ.get("ROCE_ICRC_LIB", "default")
    for name in cases:
        buf, offs, lens = make_case(name)
        n = offs.size
        want, _ = oracle_batch(buf, offs, lens)
        trail = offs.astype(np.int64) + lens.astype(np.int64) - 4
        buf[(trail[:, None] + np.arange(4)[None, :]).reshape(-1)] = want.view(np.uint8)
        d = torch.from_numpy(buf).cuda()
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        dl = torch.from_numpy(lens.view(np.int32)).cuda()
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        cov = float(synth.covered_bytes(lens))
        alg = float(lens.astype(np.int64).sum()) + 12.0 * n  # frames + descriptors read
        for mode in ("compute", "verify"):
            if mode == "compute":
                fn = lambda: eng.compute_batch_dev(d, do, dl, n, out, stream=s.cuda_stream)  # noqa: E731
            else:
                fn = lambda: eng.verify_batch_dev(d, do, dl, n, ok, stream=s.cuda_stream)  # noqa: E731
            fn()
            s.synchronize()
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                fn()
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e-3)
            t = float(np.median(ts))
            if mode == "compute":
                bad = int((out.cpu().numpy().view(np.uint32) != want).sum())
            else:
                bad = int((ok.cpu().numpy() != 1).sum())
            wr = 4.0 * n if mode == "compute" else 1.0 * n
            print(json.dumps({"lib": lib, "case": name, "mode": mode, "n": n,
                              "ms": round(t * 1e3, 4), "GiBps": round(cov / t / 2**30, 1),
                              "GBps_alg": round((alg + wr) / t / 1e9, 1),
                              "mismatches": bad}), flush=True)
        del d, do, dl, out, ok
        torch.cuda.empty_cache()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cases", default="u4,u12,u60,mix,cfg3")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("libs", nargs="*")
    args = ap.parse_args()
    cases = args.cases.split(",")
    if args.child:
        child(cases, args.reps)
        return
    for rnd in range(args.rounds):
        for lib in args.libs:
            env = dict(os.environ, ROCE_ICRC_LIB=str(Path(lib).resolve()))
            r = subprocess.run([sys.executable, __file__, "--child", "--cases", args.cases,
                                "--reps", str(args.reps)], env=env, timeout=600)
            if r.returncode != 0:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()

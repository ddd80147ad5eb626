#!/usr/bin/env python3
"""Speed ratios kept out of the `-m gpu` correctness gate (bench evidence).

Two numbers the test suite used to assert, now measured here and kept under
profiles/ (round 5 verdict, item 5: a contended box must not turn a
bit-exact suite red):

* ``ragged``: a device-resident batch of 2^22 packed ACK frames
  (src/roce_rq.py:767-853) on the COMPACT and the SORTED ragged kernel, named
  per launch (ABI 5), K launches each between one event pair, three
  alternating rounds; every word checked against the C oracle.
* ``service``: scripts/svc_contention.py -- cfg2-shaped batches beside K
  threads calling ricrc_icrc back to back (src/sanity_side.py:383's pool).

usage: python scripts/perf_ratios.py [--out FILE] [--packets N]
prints (and writes) one JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "roce-sim_amd"), str(ROOT / "oracle"), str(ROOT / "tests"),
                str(ROOT / "scripts")]


def ragged(packets: int, launches: int = 10, rounds: int = 3) -> dict:
    import torch

    from conftest import oracle_batch  # checker only
    from roce_icrc import IcrcEngine, synth
    from roce_icrc import engine as E

    buf, offs, lens = synth.mixed_mtu_frames(packets, mtus=(4,), opcode=0x11, seed=8)
    want, _ = oracle_batch(buf, offs, lens)
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(packets, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    eng = IcrcEngine(0)
    names = {E.RAGGED_COMPACT: "compact", E.RAGGED_SORTED: "sorted"}
    ms = {v: [] for v in names}
    exact = {v: True for v in names}
    try:
        for _ in range(rounds):
            for v in names:
                eng.set_ragged_variant(v)
                for _ in range(3):  # warm
                    eng.compute_batch_dev(d, do, dl, packets, out, stream=s.cuda_stream)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for _ in range(launches):
                    eng.compute_batch_dev(d, do, dl, packets, out, stream=s.cuda_stream)
                b.record(s)
                s.synchronize()
                assert eng.last_ragged_variant() == v
                ms[v].append(a.elapsed_time(b) / launches)
                exact[v] &= bool((out.cpu().numpy().view(np.uint32) == want).all())
                out.zero_()
    finally:
        eng.close()
    med = {names[v]: round(float(np.median(x)), 4) for v, x in ms.items()}
    return {"packets": packets, "frame_bytes": int(lens[0]), "launches_per_round": launches,
            "rounds": rounds, "kernel_ms_median": med,
            "kernel_ms_per_round": {names[v]: [round(t, 4) for t in x] for v, x in ms.items()},
            "compact_over_sorted": round(med["compact"] / med["sorted"], 4),
            "bit_exact": {names[v]: e for v, e in exact.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 22)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import svc_contention
    t0 = time.perf_counter()
    res = {"ragged": ragged(a.packets)}
    print("ragged", json.dumps(res["ragged"]), flush=True)
    res["service"] = svc_contention.run(packets=1 << 18, reps=40, ks=(0, 1, 4, 10))
    res["s"] = round(time.perf_counter() - t0, 1)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(line + "\n")
    ok = all(res["ragged"]["bit_exact"].values()) and all(
        v["batch_bit_exact"] and not v["errors"] for v in res["service"]["per_k"].values())
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()

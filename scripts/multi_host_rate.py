#!/usr/bin/env python3
"""Host-inclusive rate of the multi-device C-ABI split.

ricrc_compute_batch_multi / ricrc_verify_batch_multi take one host batch
(pageable numpy memory, as a simulator would hand it over), gather each
shard through the context's pinned staging blocks, copy, run the ragged
kernel and scatter the answers (icrc_capi.cpp, multi_shard).  This times
them with K contexts -- on distinct devices when the box has them, else K
contexts on device 0 (host threads and PCIe copies in parallel, one GPU) --
next to ricrc_compute_batch on one context.  GiB/s of covered bytes
(SURVEY.md section 8(d)), best of R calls; every answer checked against the
C oracle (checker only).

usage: python scripts/multi_host_rate.py [--packets N] [--reps R] [--ks 1,2,4,8]
prints one JSON line per (workload, api, K).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "roce-sim_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", default="1,2,4,8")
    args = ap.parse_args()

    from conftest import oracle_batch  # checker only
    from roce_icrc import IcrcEngine, compute_batch_multi, synth, verify_batch_multi
    from roce_icrc import engine as E

    ndev = E.device_count()
    n = args.packets
    work = {}
    buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
    work["cfg2_4KiB"] = (buf, np.arange(n, dtype=np.uint64) * np.uint64(stride),
                         np.full(n, flen, np.uint32))
    work["cfg3_mixed"] = synth.mixed_mtu_frames(n, seed=synth.SEED_CFG3)
    for name, (buf, offs, lens) in work.items():
        want, _ = oracle_batch(buf, offs, lens)
        for i in range(n):  # stamp the trailers: verify then accepts every frame
            e = int(offs[i]) + int(lens[i])
            buf[e - 4:e] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
        cov = synth.covered_bytes(lens)
        for k in [int(x) for x in args.ks.split(",")]:
            devs = [d % ndev for d in range(k)] if ndev > 1 else [0] * k
            engines = [IcrcEngine(d) for d in devs]
            try:
                calls = {"compute_batch_multi": lambda: compute_batch_multi(engines, buf, offs, lens),
                         "verify_batch_multi": lambda: verify_batch_multi(engines, buf, offs, lens)}
                if k == 1:
                    calls["compute_batch"] = lambda: engines[0].compute_batch(buf, offs, lens)
                for api, fn in calls.items():
                    r = fn()
                    icrc = r[1] if api.startswith("verify") else r[0]
                    mism = int((icrc != want).sum())
                    if api.startswith("verify"):
                        mism += int((~r[0]).sum())
                    ts = []
                    for _ in range(args.reps):
                        t0 = time.perf_counter()
                        fn()
                        ts.append(time.perf_counter() - t0)
                    print(json.dumps({"workload": name, "api": api, "contexts": k,
                                      "devices": sorted(set(devs)), "packets": n,
                                      "frame_MB": round(buf.nbytes / 1e6, 1),
                                      "GiBps": round(cov / min(ts) / 2**30, 2),
                                      "ms_best": round(min(ts) * 1e3, 2),
                                      "ms_median": round(float(np.median(ts)) * 1e3, 2),
                                      "mismatches": mism}), flush=True)
            finally:
                for e in engines:
                    e.close()


if __name__ == "__main__":
    main()

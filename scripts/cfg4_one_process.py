#!/usr/bin/env python3
"""BASELINE config 4 at its stated size through the HIP path, in ONE process.

SURVEY.md 8(d) cfg4: 2^23 4 KiB-MTU packets (4140-B frames) of ONE stream
seeded 0x1C2C0004, packet i on GPU i mod 8 (src/roce.py:192-219 reads only
its own packet, so the split needs no collective).  The 8-GPU launch is the
driver's; this runs the same eight shards on whatever device 0 is:

1. the eight shards ``synth.shard_frames(2^23, r, 8)`` are built by a fork
   pool straight into one shared host block (8 x 4.34 GB), each rank's rows
   generated from its own PCG64 jump as bench.py's ranks do;
2. all eight are uploaded and held resident on device 0 together (34.7 GB of
   HBM) and each runs ``ricrc_compute_strided_dev`` -- the launch every cfg4
   rank makes -- and every one of the 2^23 words is compared with the C
   oracle (oracle_batch, the checker);
3. the same host stream, in stream order (descriptor i -> shard i mod 8,
   row i div 8), goes through ``ricrc_compute_batch_multi`` with eight
   contexts on device 0: the host-buffer split of DESIGN.md section 6, bit-exact
   against the same words; its host-inclusive GiB/s is recorded.

usage: python scripts/cfg4_one_process.py [--log2n 23] [--world 8] [--out FILE]
prints one JSON line (exit 3 on any mismatch).
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "roce-sim_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]

_JOB = None


def _build(r):
    from roce_icrc import synth
    blk, n_total, world, shard_bytes = _JOB
    region = np.frombuffer(blk, np.uint8, count=shard_bytes, offset=r * shard_bytes)
    synth.shard_frames(n_total, r, world, out=region)
    return r


def _procs() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16"))))


def run(log2n: int = 23, world: int = 8, log=print) -> dict:
    import multiprocessing as mp

    import torch

    from conftest import oracle_batch  # checker only
    from roce_icrc import IcrcEngine, synth
    from roce_icrc import engine as E

    global _JOB
    n_total = 1 << log2n
    assert n_total % world == 0
    per = n_total // world
    flen = synth.HDR + 4096 + synth.ICRC
    shard_bytes = per * flen
    t0 = time.perf_counter()
    blk = mmap.mmap(-1, world * shard_bytes)  # anonymous, shared with the fork pool
    _JOB = (blk, n_total, world, shard_bytes)
    with mp.get_context("fork").Pool(min(world, _procs())) as pool:
        done = sorted(pool.map(_build, range(world)))
    assert done == list(range(world))
    host = np.frombuffer(blk, np.uint8)
    t_gen = time.perf_counter() - t0
    log(f"built {world} shards x {per} frames in {t_gen:.1f} s", flush=True)

    t0 = time.perf_counter()
    want = [oracle_batch(host[r * shard_bytes:(r + 1) * shard_bytes], stride=flen, length=flen,
                         n=per)[0] for r in range(world)]
    t_oracle = time.perf_counter() - t0
    log(f"oracle {t_oracle:.1f} s", flush=True)

    # 2. every shard resident on device 0 at once, the rank's launch on each
    res = {"packets_total": n_total, "world": world, "packets_per_shard": per,
           "frame_bytes": flen, "seed": hex(synth.SEED_CFG4), "device": 0,
           "host_gen_s": round(t_gen, 1), "oracle_s": round(t_oracle, 1)}
    eng = IcrcEngine(0)
    s = torch.cuda.Stream()
    try:
        dev, outs = [], []
        for r in range(world):
            dev.append(torch.from_numpy(host[r * shard_bytes:(r + 1) * shard_bytes]).cuda())
            outs.append(torch.zeros(per, dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        res["resident_bytes"] = world * shard_bytes
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(world + 1)]
        ev[0].record(s)
        for r in range(world):
            eng.compute_strided_dev(dev[r], flen, flen, per, outs[r], stream=s.cuda_stream)
            ev[r + 1].record(s)
        s.synchronize()
        mism = [int((outs[r].cpu().numpy().view(np.uint32) != want[r]).sum()) for r in range(world)]
        ms = [ev[r].elapsed_time(ev[r + 1]) for r in range(world)]
        cov = per * (flen - 4)
        res["resident"] = {"mismatches_per_shard": mism,
                           "kernel_ms_per_shard": [round(x, 4) for x in ms],
                           "kernel_GiBps_per_shard": [round(cov / (x * 1e-3) / 2**30, 1) for x in ms]}
        log("resident", json.dumps(res["resident"]), flush=True)
        del dev, outs
        torch.cuda.empty_cache()
    finally:
        eng.close()

    # 3. the host stream through ricrc_compute_batch_multi, 8 contexts on device 0
    i = np.arange(n_total, dtype=np.uint64)
    offs = (i % np.uint64(world)) * np.uint64(shard_bytes) + (i // np.uint64(world)) * np.uint64(flen)
    lens = np.full(n_total, flen, np.uint32)
    engines = [IcrcEngine(0) for _ in range(world)]
    try:
        t0 = time.perf_counter()
        got, st = E.compute_batch_multi(engines, host, offs, lens)
        t_multi = time.perf_counter() - t0
    finally:
        for e in engines:
            e.close()
    want_stream = np.empty(n_total, np.uint32)
    for r in range(world):
        want_stream[r::world] = want[r]
    mm = int((got != want_stream).sum()) + int(st.any())
    cov_total = n_total * (flen - 4)
    res["multi"] = {"contexts": world, "devices": 1, "mismatches": mm, "s": round(t_multi, 2),
                    "host_inclusive_GiBps": round(cov_total / t_multi / 2**30, 1)}
    log("multi", json.dumps(res["multi"]), flush=True)
    res["pass"] = mm == 0 and not any(res["resident"]["mismatches_per_shard"])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = run(a.log2n, a.world)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(line + "\n")
    sys.exit(0 if res["pass"] else 3)


if __name__ == "__main__":
    main()

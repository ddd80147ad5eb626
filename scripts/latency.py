"""Per-call latency of the host-buffer entry points (the per-packet drop-in
path of BTH.compute_icrc, src/roce.py:192): ricrc_compute_one and small
ricrc_compute_batch / ricrc_verify_batch calls, synchronous H2D + kernel + D2H.

usage: python scripts/latency.py [--reps 300]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402


def med_us(fn, reps):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6), float(np.percentile(ts, 99) * 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    eng = IcrcEngine(0)
    sys.path.insert(0, str(ROOT / "oracle"))
    import icrc_oracle as orc  # checker only: every timed answer is compared
    for service in (1000, 0):  # the resident per-packet service, then one launch per call
        eng.set_service(service)
        for pay in (0, 64, 1024, 4096):
            buf, stride, flen = synth.uniform_frames(1, pay)
            frame = bytes(buf[:flen])
            want = orc.icrc_of_frame(frame)
            got = []
            med, p99 = med_us(lambda: got.append(eng.compute_one(frame)[0]), a.reps)
            assert set(got) == {want}, (hex(want), {hex(x) for x in got})
            # the reference's own arithmetic on this host, per frame (zlib.crc32
            # of the masked pseudo packet, src/roce.py:218), for scale
            zmed, _ = med_us(lambda: orc.icrc_of_frame(frame), a.reps)
            gpu = []
            if service:  # GPU-side share of a call (wave saw it -> result written)
                for _ in range(50):
                    eng.compute_one(frame)
                    gpu.append(eng.service_times())
            print(json.dumps({"call": "compute_one", "service_idle_us": service,
                              "frame_bytes": flen, "median_us": round(med, 2),
                              "p99_us": round(p99, 2), "calls": len(got),
                              "gpu_side_median_us": round(float(np.median([g[0] for g in gpu])), 2)
                              if gpu else None,
                              "polls_median": float(np.median([g[1] for g in gpu])) if gpu else None,
                              "cpu_restatement_median_us": round(zmed, 2)}), flush=True)
        # a call after the wave has timed out (service relaunch included)
        if service:
            import time as _t
            _t.sleep(0.01)
            t0 = time.perf_counter()
            eng.compute_one(frame)
            print(json.dumps({"call": "compute_one after idle exit", "frame_bytes": flen,
                              "us": round((time.perf_counter() - t0) * 1e6, 1)}), flush=True)
    # the context-free call (engine.icrc -> ricrc_icrc, this thread's
    # library-owned context)
    from roce_icrc import engine as E
    for pay in (0, 4096):
        buf, stride, flen = synth.uniform_frames(1, pay)
        frame = bytes(buf[:flen])
        want = orc.icrc_of_frame(frame)
        got = []
        med, p99 = med_us(lambda: got.append(E.icrc(frame)[0]), a.reps)
        assert set(got) == {want}, (hex(want), {hex(x) for x in got})
        print(json.dumps({"call": "icrc (no context)", "frame_bytes": flen,
                          "median_us": round(med, 2), "p99_us": round(p99, 2)}), flush=True)
    # bursts: up to 64 frames / 64 KiB go to the resident wave as ONE request
    # (round 3), larger batches and service 0 launch the kernels
    acks = [orc.build_frame("10.0.0.2", "10.0.0.1", 9, dict(opcode=0x11, psn=i, dqpn=5),
                            ext=orc.aeth_bytes(0, 31, i)) for i in range(64)]
    abuf = np.frombuffer(b"".join(acks), np.uint8).copy()
    aoffs = np.arange(64, dtype=np.uint64) * len(acks[0])
    alens = np.full(64, len(acks[0]), np.uint32)
    for service in (1000, 0):
        eng.set_service(service)
        cases = [("mixed-MTU", n) + synth.mixed_mtu_frames(n, seed=3) for n in (1, 4, 16, 256, 4096)]
        cases.append(("ACK", 64, abuf, aoffs, alens))
        for kind, n, buf, offs, lens in cases:
            want = np.array([orc.icrc_of_frame_at(buf, int(a_), int(b_)) for a_, b_ in zip(offs, lens)],
                            np.uint32)
            got = []
            med, p99 = med_us(lambda: got.append(eng.compute_batch(buf, offs, lens)[0]),
                              max(20, a.reps // 4))
            assert all((g == want).all() for g in got)
            zmed, _ = med_us(lambda: [orc.icrc_of_frame_at(buf, int(a_), int(b_))
                                      for a_, b_ in zip(offs, lens)], max(20, a.reps // 4))
            cov = synth.covered_bytes(lens)
            gpu = None
            if service and n <= 64:  # GPU side of a burst request (stamps land after the answers)
                g = []
                for _ in range(30):
                    eng.compute_batch(buf, offs, lens)
                    time.sleep(0.0005)
                    g.append(eng.service_times()[0])
                gpu = round(float(np.median(g)), 2)
            print(json.dumps({"call": "compute_batch", "frames": kind, "n": n, "gpu_side_median_us": gpu,
                              "service_idle_us": service, "bytes": int(lens.sum()),
                              "median_us": round(med, 2), "p99_us": round(p99, 2),
                              "GiBps": round(cov / med / 1e-6 / 2**30, 3),
                              "cpu_restatement_median_us": round(zmed, 2)}), flush=True)
            med, p99 = med_us(lambda: eng.verify_batch(buf, offs, lens), max(20, a.reps // 4))
            print(json.dumps({"call": "verify_batch", "frames": kind, "n": n,
                              "service_idle_us": service, "median_us": round(med, 2),
                              "p99_us": round(p99, 2)}), flush=True)
    eng.set_service(1000)

if __name__ == "__main__":
    main()

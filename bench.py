#!/usr/bin/env python3
"""bench.py -- device-resident RoCEv2 ICRC throughput on MI355X (BASELINE.json metric).

One step = one launch of the HIP ICRC kernel over one batch of synthetic frames
already resident in HBM.  Default workload (N=1): BASELINE config 2, 2^20 RC
SEND_MIDDLE frames with 4 KiB payloads (4140-B wire frames, compute mode).
With --gpus N (one process per GPU: under torch.distributed.run, or -- run
plainly as `python bench.py --gpus N` -- bench.py starts the N ranks itself
under torch.distributed.run as a child process) the default workload is
BASELINE config 4: ONE stream of 2^20 N frames (seed 0x1C2C0004,
2^23 packets at N = 8), packet i on rank i mod N; there is no data-path
collective, only a gloo barrier, a max-reduce of the timing (weak scaling) and
a gather of every rank's parity result.  --workload cfg3 / cfg5 run the other
BASELINE configurations (mixed-MTU verify, 64-B payloads) with the same
contract.

Every rank checks its own GPU words against the CPU restatement of
BTH.compute_icrc on a seeded sample of >= 65536 of its packets (all of them
when fewer) and the line fails (exit status 3) on any mismatch.

Printed (rank 0): ONE JSON line with the driver's keys plus
  roofline      -- achieved algorithmic GB/s of the ICRC kernel (per-launch
                   bytes / mean launch time: the K back-to-back timed launches
                   between one pair of HIP events on the launch stream, / K)
                   against the 8.0 TB/s HBM peak, and the PMC-measured
                   HBM traffic per launch when profiles/pmc_traffic_<workload>.json holds
                   it for this workload AND for this very build (the file
                   records the sha256 of the libroceicrc.so it was measured
                   on; another build gives traffic null and says why);
  cpu_baseline  -- the per-packet Python restatement of BTH.compute_icrc
                   (datenlord/roce-sim src/roce.py:192-223, zlib.crc32), timed
                   on this host's cores over a bounded sample (rank 0, over
                   its own shard at N > 1);
  parity        -- per-rank sampled bit-exactness against that restatement.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))

METRIC = "ICRC GiB/s device-resident, 4 KiB MTU packets, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
PMC_DIR = ROOT / "profiles"  # pmc_traffic_<workload>.json (scripts/pmc_traffic.py)

WORKLOADS = {
    # name: (payload bytes (0 = mixed MTU), packets per GPU, seed, description)
    "cfg2": (4096, 1 << 20, 0x1C2C0001,
             "4 KiB-MTU RC SEND_MIDDLE frames (4140 B), ICRC compute, stride 4140"),
    # one global stream, packet i on rank i mod N, 2^20 per GPU
    "cfg4": (4096, 1 << 20, 0x1C2C0004,
             "4 KiB-MTU RC SEND_MIDDLE frames (4140 B) of ONE stream seeded 0x1C2C0004, packet i "
             "on GPU i mod N, ICRC compute, stride 4140"),
    "cfg5": (64, 1 << 24, 0x1C2C0005,
             "64-B payload SEND_MIDDLE-shaped frames (108 B), ICRC compute, stride 108"),
    "cfg3": (0, 1 << 20, 0x1C2C0003,
             "mixed-MTU {256..4096} RDMA_WRITE_MIDDLE frames packed back to back, ICRC verify "
             "(GPU fault injector hits ~3/1024 frames: ICRC and payload bit flips must fail, "
             "randomised masked fields must pass)"),
    # the responder's dominant frame (src/roce_rq.py:767-776): device-resident
    # ragged batches of ACKs, the ragged COMPACT kernel
    "ack": (4, 1 << 24, 0x1C2C0007,
            "ACK frames (IPv4/UDP/BTH/AETH, 48 B) packed back to back, device-resident ragged "
            "ICRC compute (offsets + lengths in HBM)"),
    # SURVEY 8(f) rows 1 + 3: frames built on the GPU from the MR, ICRC fused
    "seg": (4096, 1 << 20, 0x1C2C0006,
            "RC SEND of 256 KiB messages from a device MR, 4 KiB PMTU (FIRST + 62 MIDDLE + "
            "LAST per WR): IPv4/UDP/BTH build, payload copy, ICRC and UDP checksum in one kernel"),
}


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: the chip's power management settles within ~30 back-to-back
    # launches (profiles/, DESIGN.md "Measurement"); 100 timed launches ~ 70 ms
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: cfg2 on one GPU, cfg4 (the 8-GPU config) with N > 1")
    ap.add_argument("--packets", type=int, default=0, help="override packets per GPU")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per packet (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# CPU baseline: the oracle's per-packet restatement (bench's only oracle use)
# ---------------------------------------------------------------------------

_CPU_JOB = None


def _cpu_chunk(se):
    import icrc_oracle as orc
    buf, offs, lens = _CPU_JOB
    s, e = se
    return np.array([orc.icrc_of_frame_at(buf, int(offs[i]), int(lens[i])) for i in range(s, e)],
                    np.uint32)


def cpu_model() -> str:
    """The host CPU's model name (record it with the core count)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> tuple[int, dict]:
    """Worker processes for the CPU baseline: every CPU this process may run
    on (sched_getaffinity), capped by a cgroup CPU quota (cpu.max) and by the
    host's declared per-job thread budget (OMP_NUM_THREADS: the GPU pool sets
    it to the box's CPU share, 16 per GPU, and its rules forbid larger pools);
    returns (procs, the counts it was derived from)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    omp = None
    try:
        omp = int(os.environ["OMP_NUM_THREADS"])
    except (KeyError, ValueError):
        pass
    procs = min(x for x in (aff, quota, omp) if x)
    return max(1, procs), {"affinity_cpus": aff, "cgroup_cpus": quota, "omp_num_threads": omp,
                           "host_cpus": os.cpu_count()}


def cpu_native_c(buf: np.ndarray, offs: np.ndarray, lens: np.ndarray, gpu_icrc: np.ndarray,
                 threads: int) -> dict:
    """The oracle's C restatement (oracle/icrc_ref.c: masked copy + slice-by-8
    CRC-32 per frame, pthreads) over the same host frames: what a native CPU
    port of BTH.compute_icrc reaches on this job's cores, beside the Python
    per-packet path the reference runs.  Whole batch, repeated to ~0.5 s."""
    import ctypes
    path = ROOT / "oracle" / "build" / "liboracle.so"
    if not path.exists():
        return {"native_c_note": f"{path.name} not built (make -C oracle)"}
    lib = ctypes.CDLL(str(path))
    lib.oracle_icrc_batch.restype = ctypes.c_int
    lib.oracle_icrc_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    n = offs.size
    out = np.zeros(n, np.uint32)
    passes, t = 0, 0.0
    while passes == 0 or (t < 0.5 and passes < 8):
        t0 = time.perf_counter()
        rc = lib.oracle_icrc_batch(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, 0, 0, n,
                                   out.ctypes.data, None, threads)
        t += time.perf_counter() - t0
        passes += 1
        if rc != 0:
            return {"native_c_note": f"oracle_icrc_batch failed ({rc})"}
    cov = int((lens.astype(np.int64) - 4).sum())
    return {"native_c_GiBps": round(passes * cov / t / 2**30, 3), "native_c_threads": threads,
            "native_c_mismatches_vs_gpu": int((out != gpu_icrc).sum())}


def cpu_baseline(buf: np.ndarray, offs: np.ndarray, lens: np.ndarray, gpu_icrc: np.ndarray):
    """Per-packet zlib restatement (oracle/, the CPU "port" baseline) on this host.

    Single process over the first ~256 MiB, then a fork pool over all packets
    (bounded: about 10 core-seconds).  Its CRCs double as a parity sample."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import multiprocessing as mp

    import icrc_oracle as orc

    n = offs.size
    cov = lens.astype(np.int64) - 4
    n1 = int(min(n, max(1, np.searchsorted(np.cumsum(lens, dtype=np.int64), 1 << 28))))
    t0 = time.perf_counter()
    one = np.array([orc.icrc_of_frame_at(buf, int(offs[i]), int(lens[i])) for i in range(n1)],
                   np.uint32)
    t1 = time.perf_counter() - t0
    procs, share = cpu_share()
    global _CPU_JOB
    _CPU_JOB = (buf, offs, lens)
    step = (n + procs * 4 - 1) // (procs * 4)
    chunks = [(s, min(n, s + step)) for s in range(0, n, step)]
    # passes over the whole batch until ~1 s of pool time (about 16 core-seconds)
    passes, tn = 0, 0.0
    with mp.get_context("fork").Pool(procs) as pool:
        while passes == 0 or (tn < 1.0 and passes < 16):
            t0 = time.perf_counter()
            parts = pool.map(_cpu_chunk, chunks)
            tn += time.perf_counter() - t0
            passes += 1
    allc = np.concatenate(parts)
    mism = int((allc != gpu_icrc).sum()) + int((one != gpu_icrc[:n1]).sum())
    native = cpu_native_c(buf, offs, lens, gpu_icrc, procs)
    mism += native.get("native_c_mismatches_vs_gpu", 0)
    c_all, c_one = int(cov.sum()), int(cov[:n1].sum())
    return {
        "value": round(passes * c_all / tn / 2**30, 4),
        "unit": "GiB/s",
        "cores": procs,
        "procs": procs,
        **share,
        "kind": "port",
        "sample": (f"Python zlib.crc32 restatement of BTH.compute_icrc per packet over the same "
                   f"host frames: {passes} pass(es) over {n} packets on a {procs}-process fork "
                   f"pool ({tn:.2f} s; {procs} = this job's CPU share, see cpu_share()); "
                   f"single core {n1} packets {c_one / t1 / 2**30:.3f} GiB/s"),
        "single_core_GiBps": round(c_one / t1 / 2**30, 4),
        # an upper estimate for a pool over every CPU of the affinity mask
        # (linear in the single-core rate; not measured)
        "single_core_x_affinity_GiBps": round(c_one / t1 / 2**30 * share["affinity_cpus"], 2),
        "cpu_model": cpu_model(),
        "parity_mismatches_vs_gpu": mism,
        **native,
    }


# ---------------------------------------------------------------------------
# Workloads
# ---------------------------------------------------------------------------


class Strided:
    """cfg2 / cfg4 / cfg5: fixed-size frames, ICRC compute."""

    mode = "compute"

    def __init__(self, torch, eng, dev, payload, n, seed, rank, world):
        from roce_icrc import synth
        self.torch, self.eng, self.n = torch, eng, n
        self.buf, self.stride, self.flen = synth.uniform_frames(
            n, payload, seed=seed if world == 1 else seed + rank, psn_start=rank, psn_step=world)
        # (cfg2 / cfg5 at N > 1: one independent replica batch per rank)
        self.offs = np.arange(n, dtype=np.uint64) * self.stride
        self.lens = np.full(n, self.flen, np.uint32)
        self.covered = n * (self.flen - 4)
        self.alg_bytes = n * self.flen  # C_i read + 4-B ICRC written
        self.d_frames = torch.from_numpy(self.buf).to(dev)
        self.out = torch.zeros(n, dtype=torch.int32, device=dev)

    def step(self, sp):
        self.eng.compute_strided_dev(self.d_frames, self.stride, self.flen, self.n, self.out,
                                     stream=sp)

    def upload(self, h_frames):
        self.d_frames.copy_(h_frames, non_blocking=True)

    def results(self):
        return self.out.cpu().numpy().view(np.uint32).copy()

    def lanes(self):
        return self.eng.lanes_for_len(self.flen)

    def check(self):
        # self-consistency on the device (the bit-exact parity against the
        # oracle is the parity leg's, the cpu_baseline leg's and the test
        # suite's): the words of the last step written into the trailers must
        # all verify, and a frame with one payload bit flipped must not.  The
        # touched bytes are restored afterwards, so the device frames are the
        # host frames again whatever runs next.
        torch, n, S, L = self.torch, self.n, self.stride, self.flen
        rows = self.d_frames[:n * S].view(n, S)
        saved = rows[:, L - 4:L].clone()
        rows[:, L - 4:L] = self.out.view(torch.uint8).view(n, 4)
        mid = n // 2
        rows[mid, L - 8] = rows[mid, L - 8] ^ 1  # last payload dword (covered, unmasked)
        ok = torch.zeros(n, dtype=torch.uint8, device=self.d_frames.device)
        self.eng.verify_strided_dev(self.d_frames, S, L, n, ok)
        okh = ok.cpu().numpy().astype(bool)
        rows[mid, L - 8] = rows[mid, L - 8] ^ 1
        rows[:, L - 4:L] = saved
        good = int(okh.sum())
        return {"words_verified": good, "frames": n, "flipped_frame_fails": bool(not okh[mid]),
                "pass": bool(good == n - 1 and not okh[mid])}


class Shard(Strided):
    """cfg4: this rank's round-robin shard (packets i = rank mod world) of ONE
    stream of n * world frames seeded 0x1C2C0004; the rank
    generates only its own packets (synth.shard_frames)."""

    def __init__(self, torch, eng, dev, payload, n, seed, rank, world):
        from roce_icrc import synth
        self.torch, self.eng = torch, eng
        self.buf, self.stride, self.flen, self.gidx = synth.shard_frames(
            n * world, rank, world, payload, seed=seed)
        self.n = n = self.gidx.size
        self.offs = np.arange(n, dtype=np.uint64) * self.stride
        self.lens = np.full(n, self.flen, np.uint32)
        self.covered = n * (self.flen - 4)
        self.alg_bytes = n * self.flen
        self.d_frames = torch.from_numpy(self.buf).to(dev)
        self.out = torch.zeros(n, dtype=torch.int32, device=dev)


class RaggedVerify:
    """cfg3: mixed-MTU frames packed back to back, ICRC verify.  Trailers are
    filled by the engine's compute path on the device (its parity is the test
    suite's job), then the GPU fault injector (ricrc_inject_faults_dev) hits
    ~3/1024 frames: ICRC bit flips and payload bit flips (must fail) and
    randomised masked fields (must pass)."""

    mode = "verify"
    FAULT_PPM = 2930  # ~3 / 1024

    def __init__(self, torch, eng, dev, payload, n, seed, rank, world):
        from roce_icrc import engine as E
        from roce_icrc import synth
        self.torch, self.eng, self.n = torch, eng, n
        self.buf, self.offs, self.lens = synth.mixed_mtu_frames(
            n, seed=seed if world == 1 else seed + rank)
        self.covered = synth.covered_bytes(self.lens)
        self.alg_bytes = self.covered + 5 * n  # C_i + 4-B trailer read, 1-B ok flag written
        self.d_frames = torch.from_numpy(self.buf).to(dev)
        self.d_offs = torch.from_numpy(self.offs.view(np.int64)).to(dev)
        self.d_lens = torch.from_numpy(self.lens.view(np.int32)).to(dev)
        self.icrc = torch.zeros(n, dtype=torch.int32, device=dev)
        self.ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        sp = torch.cuda.current_stream(dev).cuda_stream
        eng.compute_batch_dev(self.d_frames, self.d_offs, self.d_lens, n, self.icrc, stream=sp)
        trail = (self.d_offs + self.d_lens.to(torch.int64) - 4)
        idx = trail[:, None] + torch.arange(4, device=dev)[None, :]
        self.d_frames[idx.reshape(-1)] = self.icrc.view(torch.uint8).reshape(-1)
        self.fault = torch.zeros(n, dtype=torch.uint8, device=dev)
        eng.inject_faults_dev(self.d_frames, self.d_offs, self.d_lens, n, seed + 17,
                              self.FAULT_PPM, E.FAULT_ICRC | E.FAULT_PAYLOAD | E.FAULT_MASKED,
                              self.fault, stream=sp)
        torch.cuda.synchronize(dev)
        self.buf = self.d_frames.cpu().numpy()  # host copy with trailers + corruptions

    def step(self, sp):
        # verdicts only (1 B per packet); the ICRC words came from the compute path
        self.eng.verify_batch_dev(self.d_frames, self.d_offs, self.d_lens, self.n, self.ok,
                                  stream=sp)

    def upload(self, h_frames):
        self.d_frames.copy_(h_frames, non_blocking=True)

    def results(self):
        # ICRC words of the frames as they now are (faults included): the
        # compute path over the same bytes the CPU baseline reads
        sp = self.torch.cuda.current_stream(self.d_frames.device).cuda_stream
        self.eng.compute_batch_dev(self.d_frames, self.d_offs, self.d_lens, self.n, self.icrc,
                                   stream=sp)
        return self.icrc.cpu().numpy().view(np.uint32).copy()

    def lanes(self):
        return "ragged default (8 at the mixed-MTU mean)"

    def check(self):
        from roce_icrc import engine as E
        ok = self.ok.cpu().numpy().astype(bool)
        fault = self.fault.cpu().numpy()
        expect = ~np.isin(fault, [E.FAULT_ICRC, E.FAULT_PAYLOAD])
        return {"verify_ok": int(ok.sum()), "verify_failed": int((~ok).sum()),
                "faults": {"icrc": int((fault == E.FAULT_ICRC).sum()),
                           "payload": int((fault == E.FAULT_PAYLOAD).sum()),
                           "masked": int((fault == E.FAULT_MASKED).sum())},
                "verdict_matches_injected": bool((ok == expect).all()),
                "pass": bool((ok == expect).all())}


class RaggedCompute:
    """ack: ACK-sized frames packed back to back, ragged descriptors in HBM,
    ICRC compute (the responder's stream of acknowledgements)."""

    mode = "compute"

    def __init__(self, torch, eng, dev, payload, n, seed, rank, world):
        from roce_icrc import synth
        self.torch, self.eng, self.n = torch, eng, n
        # opcode 0x11 (ACKNOWLEDGE): BTH + a 4-byte AETH, 48-B frames
        self.buf, self.offs, self.lens = synth.mixed_mtu_frames(
            n, mtus=(payload,), opcode=0x11, seed=seed if world == 1 else seed + rank)
        self.covered = synth.covered_bytes(self.lens)
        # C_i read + 4-B ICRC written (48 B per ACK frame); the
        # 12-B descriptors (offset, length) are excluded and reported separately
        self.alg_bytes = self.covered + 4 * n
        self.descriptor_bytes = 12 * n
        self.d_frames = torch.from_numpy(self.buf).to(dev)
        self.d_offs = torch.from_numpy(self.offs.view(np.int64)).to(dev)
        self.d_lens = torch.from_numpy(self.lens.view(np.int32)).to(dev)
        self.out = torch.zeros(n, dtype=torch.int32, device=dev)
        # the responder knows its stream is ACKs: the compact kernel on every
        # launch (not the learned AUTO hint, which follows the last launch
        # finished before each one)
        from roce_icrc import engine as E
        eng.set_ragged_variant(E.RAGGED_COMPACT)

    def step(self, sp):
        self.eng.compute_batch_dev(self.d_frames, self.d_offs, self.d_lens, self.n, self.out,
                                   stream=sp)

    def upload(self, h_frames):
        self.d_frames.copy_(h_frames, non_blocking=True)

    def results(self):
        return self.out.cpu().numpy().view(np.uint32).copy()

    def lanes(self):
        return "ragged default (compact tiny batches: one lane per frame)"

    def check(self):
        # as Strided.check: the last step's words written into the trailers
        # all verify on the device, one frame with a payload bit flipped fails
        torch, n = self.torch, self.n
        trail = self.d_offs + self.d_lens.to(torch.int64) - 4
        idx = (trail[:, None] + torch.arange(4, device=self.d_frames.device)[None, :]).reshape(-1)
        saved = self.d_frames[idx].clone()
        self.d_frames[idx] = self.out.view(torch.uint8).reshape(-1)
        mid = n // 2
        pos = int(self.offs[mid]) + int(self.lens[mid]) - 8  # the AETH dword (covered, unmasked)
        self.d_frames[pos] ^= 1
        ok = torch.zeros(n, dtype=torch.uint8, device=self.d_frames.device)
        self.eng.verify_batch_dev(self.d_frames, self.d_offs, self.d_lens, n, ok)
        okh = ok.cpu().numpy().astype(bool)
        self.d_frames[pos] ^= 1
        self.d_frames[idx] = saved
        good = int(okh.sum())
        return {"words_verified": good, "frames": n, "flipped_frame_fails": bool(not okh[mid]),
                "pass": bool(good == n - 1 and not okh[mid])}


SEG_MSG = 256 * 1024


def _cpu_seg_chunk(se):
    import segment_oracle as so
    mr, wrs, pmtu = _CPU_JOB
    s, e = se
    return sum(len(f) - 4 for f in so.segment(mr, wrs[s:e], pmtu))


def cpu_baseline_seg(mr: np.ndarray, rec: np.ndarray, pmtu: int, frames_ok):
    """The oracle's restatement of process_send_req + scapy serialisation +
    compute_icrc per packet (segment_oracle.segment), on a bounded sample of
    the same WRs over a fork pool of this host's cores."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import multiprocessing as mp

    import segment_oracle as so

    procs, share = cpu_share()
    mv = memoryview(mr)

    def sample(nw):
        return [so.SegWR(op=int(r["op"]), mr_offset=int(r["mr_offset"]), length=int(r["length"]),
                    psn=int(r["psn"]), dqpn=int(r["dqpn"]), src_ip=int(r["src_ip"]),
                    dst_ip=int(r["dst_ip"]), sport=int(r["sport"]), flags=int(r["flags"]),
                    imm=int(r["imm"])) for r in rec[:nw]]

    # calibrate on one WR, then size the sample for about 10 s of pool time
    t0 = time.perf_counter()
    so.segment(mv, sample(1), pmtu)
    t1 = time.perf_counter() - t0
    nw = int(min(rec.size, max(procs, 10.0 * procs / max(t1, 1e-6))))
    wrs = sample(nw)
    global _CPU_JOB
    _CPU_JOB = (mv, wrs, pmtu)
    step = max(1, nw // (4 * procs))
    chunks = [(i, min(nw, i + step)) for i in range(0, nw, step)]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(procs) as pool:
        cov = sum(pool.map(_cpu_seg_chunk, chunks))
    tn = time.perf_counter() - t0
    # parity sample: the first WR's frames, oracle vs GPU
    want = so.segment(mv, wrs[:1], pmtu)
    mism = sum(int(not frames_ok(p, f)) for p, f in enumerate(want))
    return {
        "value": round(cov / tn / 2**30, 4),
        "unit": "GiB/s",
        "cores": procs,
        "procs": procs,
        **share,
        "kind": "port",
        "sample": (f"Python restatement of process_send_req + IPv4/UDP/BTH serialisation + "
                   f"zlib ICRC per packet (oracle/segment_oracle.py): {nw} WRs = "
                   f"{nw * (SEG_MSG // pmtu)} packets on a {procs}-process fork pool ({tn:.2f} s)"),
        "cpu_model": cpu_model(),
        "parity_mismatches_vs_gpu": mism,
    }


class Segment:
    """seg: MR -> frames on the GPU (ricrc_segment_dev), ICRC fused."""

    mode = "segment"

    def __init__(self, torch, eng, dev, payload, n, seed, rank, world):
        from roce_icrc import engine as E
        self.torch, self.eng, self.pmtu = torch, eng, payload
        per = SEG_MSG // payload
        nwr = max(1, n // per)
        rng = np.random.Generator(np.random.PCG64(seed if world == 1 else seed + rank))
        self.mr = rng.integers(0, 256, nwr * SEG_MSG, dtype=np.uint8)
        rec = E.seg_wrs(nwr)
        rec["op"] = E.SEG_SEND
        rec["mr_offset"] = np.arange(nwr, dtype=np.uint64) * SEG_MSG
        rec["length"] = SEG_MSG
        rec["psn"] = (np.arange(nwr, dtype=np.uint64) * per) % (1 << 24)
        rec["dqpn"] = 0x11
        rec["src_ip"], rec["dst_ip"] = 0x0A010130, 0x0A01010F
        rec["sport"] = 2
        rec["flags"] = E.SEG_SIGNALED
        self.n, self.slot = E.segment_plan(rec, payload)
        self.rec = rec
        flen = 40 + payload + 4
        self.covered = self.n * (flen - 4)
        # MR payload read + frames written + lens and ICRCs written
        self.alg_bytes = nwr * SEG_MSG + self.n * flen + 8 * self.n
        self.d_mr = torch.from_numpy(self.mr).to(dev)
        self.d_wrs = torch.from_numpy(rec.view(np.uint8)).to(dev)
        self.d_frames = torch.empty(self.n * self.slot, dtype=torch.uint8, device=dev)
        self.d_lens = torch.empty(self.n, dtype=torch.int32, device=dev)
        self.out = torch.empty(self.n, dtype=torch.int32, device=dev)

    def step(self, sp):
        self.eng.segment_dev(self.d_mr, self.mr.size, self.d_wrs, self.rec.size, self.pmtu, self.n,
                             self.d_frames, self.slot, self.d_lens, self.out, stream=sp)

    def results(self):
        return self.out.cpu().numpy().view(np.uint32).copy()

    def lanes(self):
        return self.eng.lanes_for_len(self.slot - 192)

    def frames_ok(self, pk=None):
        """Checker for the frames of packets `pk` (default: WR 0's): (i, frame)
        -> packet pk[i]'s slot and length equal the oracle's frame."""
        torch = self.torch
        torch.cuda.synchronize()
        if pk is None:
            pk = np.arange(min(self.n, SEG_MSG // self.pmtu))
        idx = torch.from_numpy(np.asarray(pk, np.int64)).to(self.d_frames.device)
        fr = self.d_frames.view(self.n, self.slot).index_select(0, idx).cpu().numpy()
        lens = self.d_lens.index_select(0, idx).cpu().numpy()
        return lambda i, f: lens[i] == len(f) and fr[i, : len(f)].tobytes() == f

    def check(self):
        from roce_icrc import engine as E
        # every frame verifies (the ICRC verify kernel over the built slots)
        torch = self.torch
        dev = self.d_frames.device
        offs = torch.arange(self.n, dtype=torch.int64, device=dev) * self.slot
        ok = torch.empty(self.n, dtype=torch.uint8, device=dev)
        self.eng.verify_batch_dev(self.d_frames, offs, self.d_lens, self.n, ok)
        torch.cuda.synchronize()
        nv, lens_ok = int(ok.sum()), bool((self.d_lens > 0).all())
        return {"frames_verified": nv, "frames": self.n, "lens_ok": lens_ok,
                "pass": bool(nv == self.n and lens_ok)}


PARITY_SAMPLE = 1 << 16  # packets per rank checked against the CPU restatement


def parity_leg(W, gpu_icrc: np.ndarray, seed: int) -> dict:
    """This rank's GPU ICRC words against the oracle's per-packet restatement
    of BTH.compute_icrc (src/roce.py:192-223) on a seeded sample of its
    packets (all of them when there are fewer than PARITY_SAMPLE); for
    segmentation, the whole frames and words of a seeded sample of WRs
    (PARITY_SAMPLE packets' worth) against segment_oracle.  Oracle use is
    confined to this checker."""
    sys.path.insert(0, str(ROOT / "oracle"))
    t0 = time.perf_counter()
    if isinstance(W, Segment):
        import segment_oracle as so
        per = SEG_MSG // W.pmtu
        nwr = W.rec.size
        kw = min(nwr, max(1, PARITY_SAMPLE // per))
        widx = (np.sort(np.random.default_rng(seed).choice(nwr, size=kw, replace=False)) if kw < nwr
                else np.arange(nwr))
        # the plan packs WR w's packets at w * per (equal-length WRs)
        pk = (widx[:, None] * per + np.arange(per)[None, :]).reshape(-1)
        ok = W.frames_ok(pk)
        wrs = [so.SegWR(op=int(r["op"]), mr_offset=int(r["mr_offset"]), length=int(r["length"]),
                        psn=int(r["psn"]), dqpn=int(r["dqpn"]), src_ip=int(r["src_ip"]),
                        dst_ip=int(r["dst_ip"]), sport=int(r["sport"]), flags=int(r["flags"]),
                        imm=int(r["imm"])) for r in W.rec[widx]]
        want = so.segment(memoryview(W.mr), wrs, W.pmtu)
        assert len(want) == pk.size
        mism = sum(int(not ok(i, f)) for i, f in enumerate(want))
        mism += sum(int(gpu_icrc[p]) != int.from_bytes(f[-4:], "little") for p, f in zip(pk, want))
        return {"sampled": len(want), "mismatches": mism,
                "what": f"whole frames + ICRC words of {kw} seeded WRs",
                "s": round(time.perf_counter() - t0, 2)}
    import icrc_oracle as orc
    n = gpu_icrc.size
    k = min(n, PARITY_SAMPLE)
    idx = (np.sort(np.random.default_rng(seed).choice(n, size=k, replace=False)) if k < n
           else np.arange(n))
    want = np.array([orc.icrc_of_frame_at(W.buf, int(W.offs[i]), int(W.lens[i])) for i in idx],
                    np.uint32)
    return {"sampled": int(k), "mismatches": int((want != gpu_icrc[idx]).sum()),
            "what": "ICRC words of a seeded packet sample", "s": round(time.perf_counter() - t0, 2)}


def lib_sha256() -> str:
    from roce_icrc import engine as E
    return hashlib.sha256(E.library_path().read_bytes()).hexdigest()


def pmc_traffic(workload: str, n: int) -> tuple[int | None, str]:
    """PMC HBM traffic per launch from profiles/pmc_traffic_<workload>.json,
    only when that file was measured on THIS libroceicrc.so (sha256) and this
    batch size; else (None, why)."""
    pmc_file = PMC_DIR / f"pmc_traffic_{workload}.json"
    if not pmc_file.exists():
        return None, f"{pmc_file.name} absent"
    try:
        pmc = json.loads(pmc_file.read_text())
    except (ValueError, OSError) as e:
        return None, f"{pmc_file.name} unreadable ({e})"
    if pmc.get("workload") != workload or pmc.get("packets") != n:
        return None, f"{pmc_file.name} is for {pmc.get('workload')} x {pmc.get('packets')} packets"
    sha = lib_sha256()
    if pmc.get("lib_sha256") != sha:
        return None, (f"{pmc_file.name} was measured on libroceicrc.so "
                      f"{(pmc.get('lib_sha256') or 'unrecorded')[:12]}, this build is {sha[:12]}: "
                      "not this build's traffic")
    return pmc.get("traffic_bytes_per_launch"), f"{pmc_file.name}, same build (sha256 {sha[:12]})"


CEIL_MIN_S = float(os.environ.get("ROCE_ICRC_CEIL_S", "0.08"))  # ceiling series length (s)


def enqueue_ceiling(torch, eng, W, stream, sp, dev):
    """Measured HBM ceiling on the same buffers: STREAM read of the frame
    buffer (16-B nt loads, one workgroup per CU sweeping a contiguous chunk,
    the ICRC kernels' geometry), or for segmentation the STREAM copy of the MR
    into the frame buffer (read + write bytes): a back-to-back series of
    >= CEIL_MIN_S, ENQUEUED without a final synchronisation so the warm-up
    steps follow it with no idle gap (see main()).  Returns a function that,
    after the stream has been synchronised, gives (key, GB/s, times)."""
    if isinstance(W, Segment):
        nb = W.mr.size // 16 * 16
        key, nbytes = "stream_copy_GBps", 2 * nb

        def launch():
            eng.stream_copy_dev(W.d_mr, W.d_frames, nb, stream=sp)
    else:
        sink = torch.zeros(4, dtype=torch.int32, device=dev)
        nb = W.d_frames.numel() // 16 * 16
        key, nbytes = "stream_read_GBps", nb

        def launch():
            eng.stream_read_dev(W.d_frames, nb, sink, stream=sp)
    launch()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    launch()
    torch.cuda.synchronize(dev)
    k = int(min(400, max(20, CEIL_MIN_S / max(time.perf_counter() - t0, 1e-5))))
    # timed as the ICRC launches are: back to back between one pair of events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        launch()
    e1.record(stream)

    def result():
        t = e0.elapsed_time(e1) * 1e-3 / k
        return key, nbytes / t / 1e9, [t] * k
    return result


def gather_ranks(dist, world: int, rank: int, device: int, wall_s: float, kern_s, covered: int):
    """Per-rank timing (per-GPU and aggregate rates):
    every rank's own wall time of the K timed steps, kernel mean and covered
    bytes, gathered (gloo) beside the MAX-reduce that gives `value`; rank
    order."""
    mine = {"rank": rank, "device": device, "wall_s": float(wall_s),
            "kernel_ms": float(np.mean(kern_s)) * 1e3, "covered": int(covered)}
    if world == 1:
        return [mine]
    ranks = [None] * world
    dist.all_gather_object(ranks, mine)
    return sorted(ranks, key=lambda r: r["rank"])


def rank_fields(ranks, steps: int) -> dict:
    """The line's per-rank keys: each rank's covered bytes of its K steps over
    its own wall time (GiB/s), its kernel mean (ms) and the rate over that
    mean, and the device it ran on.  (The slowest rank sets the aggregate: a
    slow rank or XCD shows here, not in the MAX alone.)"""
    return {
        "per_rank_GiBps": [round(r["covered"] * steps / r["wall_s"] / 2**30, 3) for r in ranks],
        "per_rank_kernel_ms": [round(r["kernel_ms"], 4) for r in ranks],
        "per_rank_kernel_GiBps": [round(r["covered"] / (r["kernel_ms"] * 1e-3) / 2**30, 3)
                                  for r in ranks],
        "per_rank_device": [r["device"] for r in ranks],
    }


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run WITHOUT a launcher (no WORLD_SIZE in the
    environment): start the N ranks under torch.distributed.run as a child
    process -- one process per GPU, 127.0.0.1 rendezvous -- and return its exit
    status.  Called before anything touches torch or the GPU (the parent never
    initialises a device, and never execs: the child is a separate process).
    Rank 0 of the child prints the JSON line on the inherited stdout."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), str(Path(__file__).resolve()), *sys.argv[1:]]
    print(f"[bench] --gpus {n} without a launcher: starting {n} ranks under "
          "torch.distributed.run", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env, cwd=str(ROOT))


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        # a launcher that started a different number of ranks than --gpus asks
        # for would print a line for the wrong N: refuse
        print(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks",
              file=sys.stderr, flush=True)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # ROCE_ICRC_BENCH_DEVICE pins every rank to one device: a rehearsal of the
    # N-rank path on a 1-GPU box (never set by the driver's scaling runs)
    local = int(os.environ.get("ROCE_ICRC_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    from roce_icrc import IcrcEngine

    eng = IcrcEngine(local, lanes=args.lanes)
    if args.workload is None:
        args.workload = "cfg2" if world == 1 else "cfg4"
    payload, n_default, seed, desc = WORKLOADS[args.workload]
    n = args.packets or n_default
    dev = torch.device("cuda", local)
    W = {"cfg3": RaggedVerify, "seg": Segment, "cfg4": Shard, "ack": RaggedCompute}.get(
        args.workload, Strided)(
        torch, eng, dev, payload, n, seed, rank, world)
    n = W.n
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    # The measured HBM ceiling (STREAM read of the same frame buffer, or the
    # STREAM copy for segmentation) is enqueued FIRST and the warm-up steps
    # right behind it, with no synchronisation in between: when the ICRC
    # kernels start on a GPU that has been idle for more than a few ms, the
    # chip's power management pulls the shader clock from ~2.1 GHz down to
    # ~1.1 GHz for launches 3-10 and takes ~50 launches to recover (up to 25 %
    # slower launches); coming straight from another HBM-saturating kernel
    # they do not dip (measured: profiles/r02_transient.txt).  The timed steps
    # are unchanged.
    #
    # The K timed launches go back to back between ONE pair of HIP events on
    # the launch stream; the mean launch duration is their elapsed time / K
    # (inter-launch gaps included).  An event pair around every launch -- the
    # form up to round 5 -- costs ~6 us per step of wall time and ~1.5 us of
    # every bracketed launch (cfg2 629.8 vs 622.9 us per step, cfg5 294.6 vs
    # 289.4; profiles/r05/step_gap_r05.txt); ROCE_ICRC_BENCH_TRACE keeps that
    # form for per-launch times.
    trace = bool(os.environ.get("ROCE_ICRC_BENCH_TRACE"))
    new_ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    evs = [(new_ev(), new_ev()) for _ in range(args.steps)] if trace else []
    wev = [(new_ev(), new_ev()) for _ in range(args.warmup)] if trace else []
    ev0, ev1 = new_ev(), new_ev()
    ceiling = enqueue_ceiling(torch, eng, W, stream, sp, dev)
    for i in range(args.warmup):
        if trace:
            wev[i][0].record(stream)
        W.step(sp)
        if trace:
            wev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        if trace:
            evs[i][0].record(stream)
        W.step(sp)
        if trace:
            evs[i][1].record(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t_local = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kern_s = ([a.elapsed_time(b) * 1e-3 for a, b in evs] if trace
              else [ev0.elapsed_time(ev1) * 1e-3 / args.steps] * args.steps)
    # the ragged kernel variant the timed launches ran (the last launch's: the
    # variant is fixed per launch on the host, include/roce_icrc.h)
    ragged_kernel = None
    if isinstance(W, (RaggedVerify, RaggedCompute)):
        ragged_kernel = {1: "compact", 2: "sorted"}.get(
            eng.last_ragged_variant(), "none")
    ceil_key, ceil_gbps, ceil_ts = ceiling()
    if trace:  # per-launch times (us) to stderr
        us = lambda xs: [round(x * 1e6) for x in xs]  # noqa: E731
        gap = wev[-1][1].elapsed_time(evs[0][0]) * 1e3 if wev and evs else -1.0
        print(f"[trace] rank {rank} ceiling n={len(ceil_ts)} {us(ceil_ts)}\n[trace] warmup "
              f"{us([a.elapsed_time(b) * 1e-3 for a, b in wev])}\n[trace] timed {us(kern_s)}\n"
              f"[trace] idle before the timed steps {gap:.1f} us, wall {t_local * 1e3:.3f} ms, "
              f"kernels {sum(kern_s) * 1e3:.3f} ms", file=sys.stderr, flush=True)
    t = torch.tensor([t_local], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t[0])
    ranks = gather_ranks(dist, world, rank, local, t_local, kern_s, W.covered)
    gpu_icrc = W.results()
    checks = W.check()
    parity = parity_leg(W, gpu_icrc, seed + 101 * rank)
    parity["rank"] = rank
    parities = [parity]
    if world > 1:
        parities = [None] * world
        dist.all_gather_object(parities, parity)

    # host-inclusive rate: pinned H2D of the frames + kernel + D2H of the results
    e2e, e2e_note = None, None
    if not args.no_e2e and hasattr(W, "upload"):
        # every rank pins its own copy of its frames: on a node that limits
        # pinned host memory the leg is skipped (same decision on every rank)
        h_pinned = h_out = None
        try:
            h_pinned = torch.from_numpy(W.buf).pin_memory()
            h_out = torch.empty(n, dtype=torch.int32).pin_memory()
            pinned = 1.0
        except RuntimeError as ex:  # (allocation failure)
            e2e_note = f"host-inclusive leg skipped: pinning {W.buf.nbytes} B failed ({ex})"[:300]
            pinned = 0.0
        flag = torch.tensor([pinned], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if float(flag[0]) < 1.0:
            e2e_note = e2e_note or "host-inclusive leg skipped: another rank could not pin its frames"
            del h_pinned, h_out
    if e2e_note is None and not args.no_e2e and hasattr(W, "upload"):
        ts = []
        for _ in range(3):
            torch.cuda.synchronize(dev)
            if world > 1:  # every rank's PCIe transfers run together
                dist.barrier()
            t0 = time.perf_counter()
            W.upload(h_pinned)
            W.step(sp)
            h_out.copy_(W.out if hasattr(W, "out") else W.icrc, non_blocking=True)
            torch.cuda.synchronize(dev)
            te = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            if world > 1:
                dist.all_reduce(te, op=dist.ReduceOp.MAX)
            ts.append(float(te[0]))
        # whole-job host-inclusive rate: all ranks' covered bytes / slowest rank
        e2e = world * W.covered / min(ts) / 2**30
        del h_pinned, h_out

    # CPU baseline (after every timed leg): rank 0 over its own frames -- at
    # N > 1 its shard of the one cfg4 stream -- while the other ranks wait at
    # the closing barrier, so the host pool has the node's cores to itself
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        if isinstance(W, Segment):
            cpu = cpu_baseline_seg(W.mr, W.rec, W.pmtu, W.frames_ok())
        else:
            cpu = cpu_baseline(W.buf, W.offs, W.lens, gpu_icrc)
        if world > 1:
            cpu["sample"] = f"rank 0's shard ({n} packets of {n * world}): " + cpu["sample"]

    if rank == 0:
        mean_k = float(np.mean(kern_s))
        achieved = W.alg_bytes / mean_k / 1e9
        traffic, traffic_src = pmc_traffic(args.workload, n)
        value = world * W.covered * args.steps / t_max / 2**30
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (numpy PCG64 payloads, scapy-default IPv4/UDP/BTH headers)",
            "config": {
                "workload": f"{args.workload}: {desc}",
                "mode": W.mode,
                "packets_per_gpu": n,
                "covered_bytes_per_gpu": W.covered,
                "lanes_per_packet": args.lanes or W.lanes(),
                **({"ragged_kernel": ragged_kernel} if ragged_kernel else {}),
                "parallelism": f"{world} GPU(s), round-robin packet shards, no collective",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": W.alg_bytes,
                **({"descriptor_bytes_per_launch": W.descriptor_bytes,
                    "frac_with_descriptors": round((W.alg_bytes + W.descriptor_bytes) / mean_k / 1e9
                                                   / HBM_PEAK_GBPS, 4)}
                   if hasattr(W, "descriptor_bytes") else {}),
            },
            "cpu_baseline": cpu,
            "parity": {
                "vs": "oracle/ CPU restatement of BTH.compute_icrc (zlib.crc32), per rank",
                "sampled_per_rank": [p["sampled"] for p in parities],
                "mismatches_per_rank": [p["mismatches"] for p in parities],
                "what": parities[0]["what"],
                "pass": all(p["mismatches"] == 0 for p in parities),
            },
            # the aggregate / N, and every rank's own numbers (rank_fields)
            "per_gpu_GiBps": round(value / world, 3),
            **rank_fields(ranks, args.steps),
            "kernel_ms_mean": round(mean_k * 1e3, 4),
            ceil_key: round(ceil_gbps, 1),
            "end_to_end_GiBps": None if e2e is None else round(e2e, 3),
            **({"end_to_end_note": e2e_note} if e2e_note else {}),
        }
        if checks:
            line["checks"] = checks
        print(json.dumps(line), flush=True)
    failed = [k for k, bad in (("checks", checks and not checks.get("pass", True)),
                                ("cpu parity", bool(cpu and cpu.get("parity_mismatches_vs_gpu"))),
                                ("sampled parity", any(p["mismatches"] for p in parities)))
              if bad]
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if failed:  # a fast wrong answer is not a result: fail loudly
        print(f"bench: rank {rank}: {', '.join(failed)} FAILED: {checks}", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()

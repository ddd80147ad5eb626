"""ctypes binding of ``libroceicrc.so`` (include/roce_icrc.h).

This is the product path of the ICRC engine: every call below runs the HIP
kernels on a gfx950 GPU.  There is deliberately no CPU fallback -- if the
library or the GPU is missing, construction raises :class:`IcrcUnavailable`.

Reference interface replaced: ``BTH.compute_icrc`` / ``BTH.pack_icrc``
(datenlord/roce-sim src/roce.py:187-223), see include/roce_icrc.h for the
mapping of every entry point.
"""

from __future__ import annotations

import ctypes
import os
import re
import threading
from pathlib import Path

import numpy as np

LIB_NAME = "libroceicrc.so"
PKG_DIR = Path(__file__).resolve().parent
REPO_ROOT = PKG_DIR.parent.parent
HEADER = REPO_ROOT / "include" / "roce_icrc.h"

RICRC_OK = 0
PKT_BAD_LEN = 0x01
PKT_NOT_IPV4 = 0x02
PKT_NOT_UDP = 0x04
PKT_LEN_MISMATCH = 0x08
PKT_ICRC_MISMATCH = 0x10
PKT_FATAL = PKT_BAD_LEN | PKT_NOT_IPV4 | PKT_NOT_UDP
PKT_SEG_BAD = 0x20

# segmentation work-request ops and flags (RICRC_SEG_*)
SEG_SEND, SEG_SEND_WITH_IMM, SEG_SEND_WITH_INV = 0, 1, 2
SEG_RDMA_WRITE, SEG_RDMA_WRITE_WITH_IMM, SEG_READ_RESPONSE = 3, 4, 5
# header-only ops (one packet each, no MR bytes)
SEG_READ_REQUEST, SEG_COMPARE_SWAP, SEG_FETCH_ADD = 6, 7, 8
SEG_ACK, SEG_RNR_NAK, SEG_NAK, SEG_ATOMIC_ACK = 9, 10, 11, 12
SEG_NUM_OPS = 13
SEG_SIGNALED, SEG_SOLICITED = 0x1, 0x2

# fault kinds (RICRC_FAULT_*)
FAULT_ICRC, FAULT_PAYLOAD, FAULT_MASKED = 0x1, 0x2, 0x4

# ragged-kernel variants (RICRC_RAGGED_*, ABI 5)
RAGGED_AUTO, RAGGED_COMPACT, RAGGED_SORTED = 0, 1, 2

# struct ricrc_seg_wr (include/roce_icrc.h), 80 bytes, as a numpy record so
# large WR batches are built vectorised
SEG_WR_DTYPE = np.dtype([
    ("mr_offset", "<u8"), ("remote_va", "<u8"), ("swap", "<u8"), ("comp", "<u8"),
    ("length", "<u4"), ("psn", "<u4"), ("dqpn", "<u4"), ("src_ip", "<u4"), ("dst_ip", "<u4"),
    ("rkey", "<u4"), ("imm", "<u4"), ("msn", "<u4"), ("sport", "<u2"), ("op", "u1"),
    ("flags", "u1"), ("first_pkt", "<u4"), ("reserved", "<u4", (2,)),
])
assert SEG_WR_DTYPE.itemsize == 80


class IcrcUnavailable(RuntimeError):
    """The HIP ICRC engine cannot run here (library not built, no gfx950 GPU)."""


class IcrcError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed: {code} ({msg})")
        self.code = code


_c_u8p = ctypes.POINTER(ctypes.c_uint8)
_c_u32p = ctypes.POINTER(ctypes.c_uint32)
_c_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p

# name -> (restype, argtypes); must cover every function in include/roce_icrc.h
_SIGNATURES = {
    "ricrc_abi_version": (ctypes.c_int, []),
    "ricrc_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "ricrc_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "ricrc_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "ricrc_ctx_destroy": (None, [_vp]),
    "ricrc_ctx_set_lanes_per_packet": (ctypes.c_int, [_vp, ctypes.c_int]),
    "ricrc_ctx_stream": (_vp, [_vp]),
    "ricrc_ctx_set_ragged_variant": (ctypes.c_int, [_vp, ctypes.c_int]),
    "ricrc_ctx_last_ragged_variant": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "ricrc_ctx_set_service": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "ricrc_ctx_service_times": (ctypes.c_int, [_vp, _vp]),
    "ricrc_compute_one": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp, _vp]),
    "ricrc_icrc": (ctypes.c_int, [_vp, ctypes.c_size_t, _vp, _vp]),
    "ricrc_compute_batch": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_size_t, _vp, _vp, ctypes.c_uint32, _vp, _vp],
    ),
    "ricrc_verify_batch": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_size_t, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp],
    ),
    "ricrc_compute_strided": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp],
    ),
    "ricrc_compute_batch_multi": (
        ctypes.c_int,
        [_vp, ctypes.c_int, _vp, ctypes.c_size_t, _vp, _vp, ctypes.c_uint32, _vp, _vp],
    ),
    "ricrc_verify_batch_multi": (
        ctypes.c_int,
        [_vp, ctypes.c_int, _vp, ctypes.c_size_t, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp],
    ),
    "ricrc_host_register": (ctypes.c_int, [_vp, ctypes.c_size_t]),
    "ricrc_host_unregister": (ctypes.c_int, [_vp]),
    "ricrc_compute_batch_dev": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp],
    ),
    "ricrc_verify_batch_dev": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp],
    ),
    "ricrc_compute_strided_dev": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp],
    ),
    "ricrc_verify_strided_dev": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp, _vp],
    ),
    "ricrc_stream_read_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "ricrc_lanes_for_len": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "ricrc_segment_plan": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    "ricrc_segment": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, ctypes.c_size_t,
         _vp, _vp, _vp],
    ),
    "ricrc_segment_dev": (
        ctypes.c_int,
        [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _vp,
         ctypes.c_uint32, _vp, _vp, _vp, _vp],
    ),
    "ricrc_stream_copy_dev": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp]),
    "ricrc_inject_faults_dev": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
         _vp, _vp],
    ),
}

_lib = None


def library_path() -> Path:
    return Path(os.environ.get("ROCE_ICRC_LIB", str(PKG_DIR / LIB_NAME)))


def load_library() -> ctypes.CDLL:
    """Load libroceicrc.so and declare every exported signature.  Loading works
    without a GPU (tests check the exports); computing needs one."""
    global _lib
    if _lib is not None:
        return _lib
    # PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7).  Import
    # it first so this library binds to that same HIP runtime: device pointers,
    # streams and events are then shared with torch (one runtime per process).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    path = library_path()
    if not path.exists():
        raise IcrcUnavailable(
            f"{path} is not built; run `make -C roce-sim_amd` (or __graft_entry__.build())"
        )
    lib = ctypes.CDLL(str(path))
    variant = bool(os.environ.get("ROCE_ICRC_LIB"))
    for name, (res, args) in _SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue  # (an A/B build older than this entry point: calling it raises)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def header_functions(header: Path = HEADER) -> list[str]:
    """Function names declared in include/roce_icrc.h."""
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ricrc_[a-z0-9_]+)\s*\(", text)))


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int(0)
    lib.ricrc_device_count(ctypes.byref(n))
    return n.value


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags.c_contiguous:
            raise ValueError("array must be C-contiguous")
        # a writable buffer's address through ctypes.from_buffer costs a third
        # of ndarray.ctypes (0.6 vs 1.7 us, five pointers per batch call: the
        # per-call latency of small bursts is mostly this host side)
        try:
            return ctypes.addressof(ctypes.c_char.from_buffer(a))
        except (TypeError, ValueError, BufferError):  # read-only or empty
            return a.ctypes.data
    if hasattr(a, "data_ptr"):  # torch tensor (device-resident calls)
        return a.data_ptr()
    return int(a)


def _descriptors(offsets, lens) -> tuple[np.ndarray, np.ndarray]:
    """(offsets u64, lens u32) of a ragged batch; one entry per frame in each."""
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    ls = np.ascontiguousarray(lens, dtype=np.uint32)
    if offs.ndim != 1 or ls.ndim != 1 or offs.size != ls.size:
        raise ValueError(f"offsets ({offs.size}) and lens ({ls.size}) must be 1-D and the same "
                         "length")
    return offs, ls


def pack_aligned(frames) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Pack byte strings into one buffer with every frame starting on a 4-byte
    boundary (the kernels' fast path; a frame at an unaligned offset takes a
    slow path).  A datagram of odd length therefore cannot shift the frames
    after it.  Returns (buffer, offsets, lens)."""
    lens = np.fromiter((len(f) for f in frames), dtype=np.uint32, count=len(frames))
    slots = (lens.astype(np.uint64) + 3) & ~np.uint64(3)
    offs = np.zeros(len(frames), np.uint64)
    if len(frames) > 1:
        offs[1:] = np.cumsum(slots[:-1])
    buf = np.zeros(int(slots.sum()), np.uint8)
    for f, o in zip(frames, offs):
        buf[int(o):int(o) + len(f)] = np.frombuffer(f, np.uint8)
    return buf, offs, lens


def _u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(a, dtype=np.uint8)
    a = np.ascontiguousarray(a)
    if a.dtype != np.uint8:
        a = a.view(np.uint8)
    return a


_tls = threading.local()  # per-thread ctypes outputs of icrc()


def icrc(frame) -> tuple[int, int]:
    """Context-free, thread-safe drop-in for BTH.compute_icrc (src/roce.py:192):
    wire frame -> (icrc, status) through ricrc_icrc, which serves each calling
    thread from a library-owned context on the thread's current HIP device
    (the reference calls compute_icrc from a 10-thread gRPC pool,
    src/sanity_side.py:383)."""
    lib = load_library()
    o = getattr(_tls, "out", None)
    if o is None:
        o = _tls.out = (ctypes.c_uint32(0), ctypes.c_uint8(0))
        _tls.refs = (ctypes.byref(o[0]), ctypes.byref(o[1]))
    if isinstance(frame, bytes):
        ptr, n = frame, len(frame)
    else:
        f = _u8(frame)
        ptr, n = (_ptr(f) if f.size else b""), f.size
    rc = lib.ricrc_icrc(ptr, n, *_tls.refs)
    if rc != RICRC_OK:
        raise IcrcError("ricrc_icrc", rc, lib.ricrc_strerror(rc).decode())
    return o[0].value, o[1].value


class IcrcEngine:
    """One ICRC context on one GPU (one HIP stream).  Not thread-safe; use one
    engine per thread, like the C context it wraps."""

    def __init__(self, device: int = 0, lanes: int = 0):
        self.lib = load_library()
        if device_count() <= device:
            raise IcrcUnavailable(f"no HIP device {device} visible")
        ctx = _vp()
        rc = self.lib.ricrc_ctx_create(device, ctypes.byref(ctx))
        if rc != RICRC_OK or not ctx.value:
            raise IcrcUnavailable(f"ricrc_ctx_create({device}) -> {rc} ({self._msg(rc)})")
        self.ctx = ctx
        self.device = device
        self._one, self._one_st = ctypes.c_uint32(0), ctypes.c_uint8(0)  # compute_one outputs
        self._one_ref, self._one_st_ref = ctypes.byref(self._one), ctypes.byref(self._one_st)
        if lanes:
            self.set_lanes(lanes)

    # -- plumbing ---------------------------------------------------------
    def _msg(self, rc: int) -> str:
        return self.lib.ricrc_strerror(rc).decode()

    def _check(self, fn: str, rc: int) -> None:
        if rc != RICRC_OK:
            raise IcrcError(fn, rc, self._msg(rc))

    def close(self) -> None:
        if getattr(self, "ctx", None) is not None and self.ctx.value:
            self.lib.ricrc_ctx_destroy(self.ctx)
            self.ctx = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_lanes(self, lanes: int) -> None:
        self._check("ricrc_ctx_set_lanes_per_packet",
                    self.lib.ricrc_ctx_set_lanes_per_packet(self.ctx, lanes))

    def set_service(self, idle_us: int) -> None:
        """Idle timeout of the per-packet service behind compute_one (0 = off:
        one kernel launch per call)."""
        self._check("ricrc_ctx_set_service", self.lib.ricrc_ctx_set_service(self.ctx, idle_us))

    def service_times(self) -> tuple[float, int]:
        """(GPU-side microseconds, polls) of the last request the per-packet
        service answered."""
        t = np.zeros(3, np.uint64)
        self._check("ricrc_ctx_service_times", self.lib.ricrc_ctx_service_times(self.ctx, _ptr(t)))
        return float(int(t[1]) - int(t[0])) * 0.01, int(t[2])

    def set_ragged_variant(self, variant: int) -> None:
        """RAGGED_AUTO (default), RAGGED_COMPACT (the compact kernel: packed
        ACK / NAK runs streamed in 64-frame groups) or RAGGED_SORTED (the
        sorted window kernel: mixed-MTU data) for this engine's ragged
        launches (include/roce_icrc.h)."""
        self._check("ricrc_ctx_set_ragged_variant",
                    self.lib.ricrc_ctx_set_ragged_variant(self.ctx, variant))

    def last_ragged_variant(self) -> int:
        """The variant the engine's last ragged kernel launch ran
        (RAGGED_COMPACT / RAGGED_SORTED; RAGGED_AUTO before any)."""
        v = ctypes.c_int(-1)
        self._check("ricrc_ctx_last_ragged_variant",
                    self.lib.ricrc_ctx_last_ragged_variant(self.ctx, ctypes.byref(v)))
        return v.value

    def lanes_for_len(self, length: int) -> int:
        return self.lib.ricrc_lanes_for_len(self.ctx, length)

    @property
    def stream(self) -> int:
        return self.lib.ricrc_ctx_stream(self.ctx) or 0

    # -- host buffers (synchronous) ----------------------------------------
    def compute_one(self, frame) -> tuple[int, int]:
        """Drop-in for BTH.compute_icrc (src/roce.py:192): wire frame -> (icrc, status).
        One ctypes call (bytes pass without a copy; the outputs are reused
        ctypes scalars), served by the context's per-packet GPU service."""
        if isinstance(frame, bytes):
            ptr, n = frame, len(frame)
        else:
            f = _u8(frame)
            ptr, n = _ptr(f), f.size
        rc = self.lib.ricrc_compute_one(self.ctx, ptr, n, self._one_ref, self._one_st_ref)
        if rc != RICRC_OK:
            self._check("ricrc_compute_one", rc)
        return self._one.value, self._one_st.value

    def compute_batch(self, frames, offsets, lens):
        f = _u8(frames)
        offs, ls = _descriptors(offsets, lens)
        n = offs.size
        out = np.zeros(n, np.uint32)
        st = np.zeros(n, np.uint8)
        self._check("ricrc_compute_batch", self.lib.ricrc_compute_batch(
            self.ctx, _ptr(f), f.size, _ptr(offs), _ptr(ls), n, _ptr(out), _ptr(st)))
        return out, st

    def verify_batch(self, frames, offsets, lens):
        f = _u8(frames)
        offs, ls = _descriptors(offsets, lens)
        n = offs.size
        ok = np.zeros(n, np.uint8)
        out = np.zeros(n, np.uint32)
        st = np.zeros(n, np.uint8)
        self._check("ricrc_verify_batch", self.lib.ricrc_verify_batch(
            self.ctx, _ptr(f), f.size, _ptr(offs), _ptr(ls), n, _ptr(ok), _ptr(out), _ptr(st)))
        return ok.astype(bool), out, st

    def compute_strided(self, frames, stride: int, length: int, n: int):
        f = _u8(frames)
        if n and f.size < (n - 1) * stride + length:
            raise ValueError("frames buffer too small")
        out = np.zeros(n, np.uint32)
        st = np.zeros(n, np.uint8)
        self._check("ricrc_compute_strided", self.lib.ricrc_compute_strided(
            self.ctx, _ptr(f), stride, length, n, _ptr(out), _ptr(st)))
        return out, st

    # -- device-resident (torch CUDA tensors), asynchronous -----------------
    def compute_strided_dev(self, d_frames, stride, length, n, d_icrc, d_status=None, stream=None):
        self._check("ricrc_compute_strided_dev", self.lib.ricrc_compute_strided_dev(
            self.ctx, _ptr(d_frames), stride, length, n, _ptr(d_icrc), _ptr(d_status), stream))

    def verify_strided_dev(self, d_frames, stride, length, n, d_ok, d_icrc=None, d_status=None,
                           stream=None):
        self._check("ricrc_verify_strided_dev", self.lib.ricrc_verify_strided_dev(
            self.ctx, _ptr(d_frames), stride, length, n, _ptr(d_ok), _ptr(d_icrc), _ptr(d_status),
            stream))

    def compute_batch_dev(self, d_frames, d_offsets, d_lens, n, d_icrc, d_status=None,
                          stream=None):
        self._check("ricrc_compute_batch_dev", self.lib.ricrc_compute_batch_dev(
            self.ctx, _ptr(d_frames), _ptr(d_offsets), _ptr(d_lens), n, _ptr(d_icrc),
            _ptr(d_status), stream))

    def verify_batch_dev(self, d_frames, d_offsets, d_lens, n, d_ok, d_icrc=None, d_status=None,
                         stream=None):
        self._check("ricrc_verify_batch_dev", self.lib.ricrc_verify_batch_dev(
            self.ctx, _ptr(d_frames), _ptr(d_offsets), _ptr(d_lens), n, _ptr(d_ok), _ptr(d_icrc),
            _ptr(d_status), stream))

    # -- MR -> packet segmentation fused with the ICRC ------------------------
    def segment(self, mr, wrs: np.ndarray, pmtu: int):
        """Build every frame of a WR batch on the GPU (process_send_req /
        process_write_req / ReadReqCtx.commit, src/roce_sq.py:1243-1411,
        src/roce_rq.py:388-438; header-only ops: process_read_req /
        process_atomic_req src/roce_sq.py:1413-1466, process_ack /
        process_nak_* src/roce_rq.py:767-854, the atomic acknowledge of
        AtomicReqCtx.commit src/roce_rq.py:490-525), all in one launch.
        Plans ``wrs`` in place.  Returns (frames [npkts, slot] uint8, lens,
        icrc, status)."""
        m = _u8(mr)
        npkts, slot = segment_plan(wrs, pmtu)
        frames = np.zeros((npkts, slot), np.uint8)
        lens = np.zeros(npkts, np.uint32)
        icrc = np.zeros(npkts, np.uint32)
        st = np.zeros(npkts, np.uint8)
        self._check("ricrc_segment", self.lib.ricrc_segment(
            self.ctx, _ptr(m), m.size, _ptr(wrs), wrs.size, pmtu, _ptr(frames), frames.size,
            _ptr(lens), _ptr(icrc), _ptr(st)))
        return frames, lens, icrc, st

    def segment_dev(self, d_mr, mr_bytes, d_wrs, nwr, pmtu, npkts, d_frames, slot, d_lens,
                    d_icrc=None, d_status=None, stream=None):
        self._check("ricrc_segment_dev", self.lib.ricrc_segment_dev(
            self.ctx, _ptr(d_mr), mr_bytes, _ptr(d_wrs), nwr, pmtu, npkts, _ptr(d_frames), slot,
            _ptr(d_lens), _ptr(d_icrc), _ptr(d_status), stream))

    def inject_faults_dev(self, d_frames, d_offsets, d_lens, n, seed, rate_ppm, kinds,
                          d_fault_out=None, stream=None):
        """Corrupt a seed-determined subset of frames in place (RICRC_FAULT_*)."""
        self._check("ricrc_inject_faults_dev", self.lib.ricrc_inject_faults_dev(
            self.ctx, _ptr(d_frames), _ptr(d_offsets), _ptr(d_lens), n, seed, rate_ppm, kinds,
            _ptr(d_fault_out), stream))

    def stream_copy_dev(self, d_src, d_dst, nbytes, stream=None):
        self._check("ricrc_stream_copy_dev", self.lib.ricrc_stream_copy_dev(
            self.ctx, _ptr(d_src), _ptr(d_dst), nbytes, stream))

    def stream_read_dev(self, d_buf, nbytes, d_sink, stream=None):
        self._check("ricrc_stream_read_dev", self.lib.ricrc_stream_read_dev(
            self.ctx, _ptr(d_buf), nbytes, _ptr(d_sink), stream))


def seg_wrs(n: int) -> np.ndarray:
    """A zeroed array of n ``ricrc_seg_wr`` records."""
    return np.zeros(n, dtype=SEG_WR_DTYPE)


def segment_plan(wrs: np.ndarray, pmtu: int) -> tuple[int, int]:
    """Util.compute_wr_pkt_num over a WR batch (host only, no GPU): fills
    ``wrs['first_pkt']`` in place, returns (total packets, slot bytes)."""
    if wrs.dtype != SEG_WR_DTYPE or not wrs.flags.c_contiguous:
        raise ValueError("wrs must be a C-contiguous SEG_WR_DTYPE array")
    lib = load_library()
    n = ctypes.c_uint32(0)
    slot = ctypes.c_uint32(0)
    rc = lib.ricrc_segment_plan(_ptr(wrs), wrs.size, pmtu, ctypes.byref(n), ctypes.byref(slot))
    if rc != RICRC_OK:
        raise IcrcError("ricrc_segment_plan", rc, lib.ricrc_strerror(rc).decode())
    return n.value, slot.value


def compute_batch_multi(engines: list[IcrcEngine], frames, offsets, lens):
    """Round-robin split over several GPUs (packet i -> engines[i % len])."""
    lib = load_library()
    f = _u8(frames)
    offs, ls = _descriptors(offsets, lens)
    n = offs.size
    arr = (_vp * len(engines))(*[e.ctx.value for e in engines])
    out = np.zeros(n, np.uint32)
    st = np.zeros(n, np.uint8)
    rc = lib.ricrc_compute_batch_multi(arr, len(engines), _ptr(f), f.size, _ptr(offs), _ptr(ls),
                                       n, _ptr(out), _ptr(st))
    if rc != RICRC_OK:
        raise IcrcError("ricrc_compute_batch_multi", rc, lib.ricrc_strerror(rc).decode())
    return out, st


def verify_batch_multi(engines: list[IcrcEngine], frames, offsets, lens):
    """Receive-side round-robin split (packet i -> engines[i % len]): what
    RoCEv2.recv_pkts (src/roce_v2.py:327-372) would call with one received
    batch on a node of several GPUs.  Returns (ok, icrc, status)."""
    lib = load_library()
    f = _u8(frames)
    offs, ls = _descriptors(offsets, lens)
    n = offs.size
    arr = (_vp * len(engines))(*[e.ctx.value for e in engines])
    ok = np.zeros(n, np.uint8)
    out = np.zeros(n, np.uint32)
    st = np.zeros(n, np.uint8)
    rc = lib.ricrc_verify_batch_multi(arr, len(engines), _ptr(f), f.size, _ptr(offs), _ptr(ls),
                                      n, _ptr(ok), _ptr(out), _ptr(st))
    if rc != RICRC_OK:
        raise IcrcError("ricrc_verify_batch_multi", rc, lib.ricrc_strerror(rc).decode())
    return ok.astype(bool), out, st


def pack_icrc(icrc: int) -> bytes:
    """BTH.pack_icrc (src/roce.py:187-190): the wire bytes are little-endian."""
    return int(icrc & 0xFFFFFFFF).to_bytes(4, "little")

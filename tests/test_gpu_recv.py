"""GPU: the receive loop with the GPU ICRC verify (roce_icrc.recv.RecvLoop):
a responder-side burst (4 KiB data frames, ACKs, NAKs, read responses) from a
capture file and from memory, corrupted frames dropped, the rest dispatched
like recv_pkts (src/roce_v2.py:327-372); on a box that allows raw sockets,
the loopback path too."""
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import icrc_oracle as o  # noqa: E402  (checker only)
import segment_oracle as SO  # noqa: E402
from roce_icrc import recv as RV  # noqa: E402
from roce_icrc import roce as R  # noqa: E402


def _burst(n=300):
    """Frames the simulator exchanges: data (up to 4 KiB), ACK/NAK, atomic
    acks, read requests; every 17th with one covered bit flipped."""
    rng = np.random.default_rng(8)
    mr = rng.integers(0, 256, 64 * 4096, dtype=np.uint8).tobytes()
    wrs, bad = [], set()
    for i in range(n):
        op = int(rng.integers(0, SO.ATOMIC_ACK + 1))
        ln = int(rng.integers(0, 2 * 4096)) if op < SO.READ_REQUEST else 64
        wrs.append(SO.SegWR(op=op, mr_offset=int(rng.integers(0, len(mr) - ln)), length=ln,
                            psn=i * 4, dqpn=0x40 + i % 3, src_ip=0x7F000001, dst_ip=0x7F000001,
                            sport=0x11, msn=i, imm=3))
    frames = SO.segment(mr, wrs, 4096)
    for k in range(0, len(frames), 17):
        f = bytearray(frames[k])
        f[len(f) // 2] ^= 0x20
        frames[k] = bytes(f)
        bad.add(k)
    return frames, bad


def test_gpu_recv_loop_from_memory_and_capture(engine, tmp_path):
    R.set_engine(engine)
    frames, bad = _burst()
    good = [f for k, f in enumerate(frames) if k not in bad]
    p = tmp_path / "burst.pcap"
    RV.write_pcap(p, frames, linktype=RV.LINKTYPE_ETHERNET)
    for src in (RV.ListSource(frames), RV.PcapSource(p)):
        loop = RV.RecvLoop(src, batch=128, keep_dropped=True)
        pk = loop.packets(len(good))
        assert len(pk) == len(good)
        for b, f in zip(pk, good):
            assert bytes(b.build()) == f[28:], "BTH bytes of the delivered frame"
        assert loop.stats.icrc_dropped == len(bad)
        assert sorted(loop.stats.dropped_frames) == sorted(frames[k] for k in bad)
        assert loop.stats.gpu_calls == (len(frames) + 127) // 128
        with pytest.raises(socket.timeout):
            loop.recv_pkts(1)


def test_gpu_recv_loop_qpn_filter(engine):
    R.set_engine(engine)
    frames, bad = _burst(120)
    loop = RV.RecvLoop(RV.ListSource(frames), batch=1000)
    want = [k for k, f in enumerate(frames) if k not in bad and int.from_bytes(f[33:36], "big") == 0x41]
    ops = loop.recv_pkts(len(want), qpn=0x41)
    assert ops == [frames[k][28] for k in want]


def test_gpu_recv_loop_raw_socket_loopback(engine):
    R.set_engine(engine)
    try:
        sink, src = RV.RawIpSink(), RV.RawSocketSource()
    except PermissionError:
        pytest.skip("raw sockets need CAP_NET_RAW on this box")
    try:
        frames, bad = _burst(60)
        sink.send(frames)
        loop = RV.RecvLoop(src, batch=256, timeout=5.0)
        good = [f for k, f in enumerate(frames) if k not in bad]
        pk = loop.packets(len(good))
        assert [bytes(b.build()) for b in pk] == [f[28:] for f in good]
        assert loop.stats.icrc_dropped == len(bad)
    finally:
        sink.close()
        src.close()


def test_gpu_recv_loop_multi_device_verifier(engine):
    """RecvLoop with its batches split over several contexts
    (roce.multi_device_verifier -> ricrc_verify_batch_multi): the same
    deliveries and drops as the one-device loop.  On a one-GPU box the
    contexts share device 0 (the split and the scatter are what is tested)."""
    from roce_icrc import IcrcEngine
    from roce_icrc.engine import device_count
    R.set_engine(engine)
    frames, bad = _burst(200)
    good = [f for k, f in enumerate(frames) if k not in bad]
    others = [IcrcEngine(d % device_count()) for d in range(1, 3)]
    try:
        loop = RV.RecvLoop(RV.ListSource(frames), batch=97, keep_dropped=True,
                           verify=R.multi_device_verifier([engine] + others))
        pk = loop.packets(len(good))
        assert [bytes(b.build()) for b in pk] == [f[28:] for f in good]
        assert loop.stats.icrc_dropped == len(bad)
        assert sorted(loop.stats.dropped_frames) == sorted(frames[k] for k in bad)
    finally:
        for e in others:
            e.close()

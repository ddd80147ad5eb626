"""CPU: the receive loop's plumbing (roce_icrc.recv) -- capture files, the
raw-socket source on loopback (no 1024-byte cap), batching, drop / skip /
dispatch like the reference's recv_pkts (src/roce_v2.py:327-372,
src/roce_rq.py:877-931).  The ICRC verdicts here come from the oracle as an
injected checker; the GPU verify is tests/test_gpu_recv.py."""
import socket

import numpy as np
import pytest

import icrc_oracle as o
from roce_icrc import recv as RV


def _frames(n=12, pay=4096, dqpn=0x21):
    rng = np.random.default_rng(3)
    return [o.build_frame("127.0.0.1", "127.0.0.1", 0x11, dict(opcode=0x01, psn=i, dqpn=dqpn + i % 2),
                          payload=rng.integers(0, 256, pay, dtype=np.uint8).tobytes())
            for i in range(n)]


def oracle_verify(frames):
    return [o.verify_frame(f) for f in frames]


def test_pcap_round_trip(tmp_path):
    fr = _frames(5) + [b"\x45" + bytes(30)]
    for lt in (RV.LINKTYPE_RAW, RV.LINKTYPE_ETHERNET):
        p = tmp_path / f"c{lt}.pcap"
        assert RV.write_pcap(p, fr, linktype=lt) == len(fr)
        src = RV.PcapSource(p)
        got = src.recv_batch(4, None) + src.recv_batch(100, None)
        assert got == fr
        with pytest.raises(socket.timeout):
            src.recv_batch(1, None)
        src.close()


def test_loop_drops_bad_icrc_skips_other_qps_and_dispatches():
    fr = _frames(12)
    fr[3] = fr[3][:100] + bytes([fr[3][100] ^ 1]) + fr[3][101:]  # ICRC must fail
    stray = o.build_frame("127.0.0.1", "127.0.0.1", 9, dict(opcode=0x01, psn=0, dqpn=0x21),
                          payload=bytes(8), dport=5000)  # not RoCE
    seen = []
    loop = RV.RecvLoop(RV.ListSource(fr[:6] + [stray] + fr[6:]), dispatch=lambda p: seen.append(p.psn) or p.opcode,
                       batch=4, verify=oracle_verify, keep_dropped=True)
    ops = loop.recv_pkts(5, qpn=0x21)  # psn 0, 2, (3 dropped), 4, 6, 8
    assert ops == [0x01] * 5 and seen == [0, 2, 4, 6, 8]
    st = loop.stats
    assert st.icrc_dropped == 1 and st.dropped_frames == [fr[3]] and st.not_roce == 1
    assert st.other_qp >= 2 and st.delivered == 5
    with pytest.raises(socket.timeout):  # the source runs dry
        loop.recv_pkts(10, qpn=0x21)


def test_npkt_zero_expects_the_timeout():
    assert RV.RecvLoop(RV.ListSource([]), verify=oracle_verify).recv_pkts(0) == []
    with pytest.raises(AssertionError):
        RV.RecvLoop(RV.ListSource(_frames(1)), verify=oracle_verify).recv_pkts(0)
    # what the reference's port-4791 socket would not see (other UDP ports)
    # and frames dropped for their ICRC do not end the wait for the timeout
    bad = _frames(2)[1]
    bad = bad[:60] + bytes([bad[60] ^ 4]) + bad[60:][1:]
    stray = o.build_frame("127.0.0.1", "127.0.0.1", 9, dict(opcode=0x01, psn=0, dqpn=0x21),
                          payload=bytes(8), dport=5000)
    loop = RV.RecvLoop(RV.ListSource([stray, bad, stray]), batch=1, verify=oracle_verify)
    assert loop.recv_pkts(0) == []
    assert loop.stats.not_roce == 2 and loop.stats.icrc_dropped == 1


def test_npkt_zero_sees_packets_an_earlier_batch_left_queued():
    """A batch larger than npkt leaves verified packets queued: the reference's
    socket would deliver the next one at once, so recv_pkts(0) asserts without
    waiting on the source (which here would only time out)."""
    fr = _frames(4)
    loop = RV.RecvLoop(RV.ListSource(fr), batch=4, verify=oracle_verify)
    assert loop.recv_pkts(1) == [0x01]  # one batch of 4 verified, 3 left queued
    with pytest.raises(AssertionError, match="should not receive"):
        loop.recv_pkts(0)


def _raw_pair():
    try:
        return RV.RawIpSink(), RV.RawSocketSource()
    except PermissionError:
        pytest.skip("raw sockets need CAP_NET_RAW")


def test_raw_socket_loopback_no_1024_byte_cap():
    """4 KiB frames sent with IP_HDRINCL to 127.0.0.1:4791 come back whole
    from the raw source (the reference's UDP socket would cut them at 1024 B),
    verify, and dispatch in order."""
    sink, src = _raw_pair()
    try:
        fr = _frames(8, pay=4096) + _frames(4, pay=64)
        sink.send(fr)
        loop = RV.RecvLoop(src, batch=64, timeout=5.0, verify=oracle_verify)
        pk = loop.packets(len(fr))
        assert [p.psn for p in pk] == [int.from_bytes(f[37:40], "big") for f in fr]
        assert loop.stats.icrc_dropped == 0 and loop.stats.delivered == len(fr)
        assert max(len(f) for f in fr) > 4000
    finally:
        sink.close()
        src.close()

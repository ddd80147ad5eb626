"""Segmentation, CPU side: the host planner of the C ABI (no GPU needed) and
the segmentation oracle's self-consistency (its frames are well-formed RoCEv2
frames that reassemble to the MR bytes)."""
from __future__ import annotations

import struct

import numpy as np
import pytest

import icrc_oracle as O
import segment_oracle as SO
from roce_icrc import engine as E
from segment_cases import all_ops_cases, lengths_for, to_records

PMTUS = (256, 512, 1024, 2048, 4096)


@pytest.mark.parametrize("pmtu", PMTUS)
def test_plan_matches_compute_wr_pkt_num(pmtu):
    rng = np.random.default_rng(pmtu)
    lens = [0, 1, pmtu - 1, pmtu, pmtu + 1] + [int(x) for x in rng.integers(0, 40000, 200)]
    rec = E.seg_wrs(len(lens))
    rec["length"] = lens
    rec["op"] = rng.integers(0, 6, len(lens))
    npkts, slot = E.segment_plan(rec, pmtu)
    counts = [SO.wr_pkt_num(n, pmtu) for n in lens]
    assert npkts == sum(counts)
    assert list(rec["first_pkt"]) == list(np.concatenate([[0], np.cumsum(counts)[:-1]]))
    assert slot % 128 == 0 and slot >= 60 + pmtu + 4 and slot - (60 + pmtu + 4) < 128


def test_plan_rejects_bad_arguments():
    rec = E.seg_wrs(2)
    with pytest.raises(E.IcrcError):
        E.segment_plan(rec, 1000)  # not an IB MTU
    rec[1]["op"] = E.SEG_NUM_OPS
    with pytest.raises(E.IcrcError):
        E.segment_plan(rec, 1024)
    big = E.seg_wrs(300)  # 300 x 2^24 packets
    big["length"] = 0xFFFFFFFF
    with pytest.raises(E.IcrcError):  # > 2^32 packets in total
        E.segment_plan(big, 256)


def test_plan_empty_batch():
    assert E.segment_plan(E.seg_wrs(0), 4096)[0] == 0


def test_seg_wr_layout_matches_header():
    """Field offsets of SEG_WR_DTYPE == struct ricrc_seg_wr (include/roce_icrc.h)."""
    offs = {name: E.SEG_WR_DTYPE.fields[name][1] for name in E.SEG_WR_DTYPE.names}
    assert offs == dict(mr_offset=0, remote_va=8, swap=16, comp=24, length=32, psn=36, dqpn=40,
                        src_ip=44, dst_ip=48, rkey=52, imm=56, msn=60, sport=64, op=66, flags=67,
                        first_pkt=68, reserved=72)
    assert E.SEG_WR_DTYPE.itemsize == 80


def test_plan_counts_header_only_ops_as_one_packet():
    """Read requests, atomics, ACK/NAKs and atomic acks are one packet each
    whatever their length field (RETH.dlen for a read request)."""
    rec = E.seg_wrs(9)
    rec["op"] = [E.SEG_SEND, E.SEG_READ_REQUEST, E.SEG_COMPARE_SWAP, E.SEG_FETCH_ADD, E.SEG_ACK,
                 E.SEG_RNR_NAK, E.SEG_NAK, E.SEG_ATOMIC_ACK, E.SEG_READ_RESPONSE]
    rec["length"] = [3000, 100000, 5, 0, 1 << 30, 7, 8, 9, 2049]
    npkts, _ = E.segment_plan(rec, 1024)
    assert npkts == 3 + 7 + 3
    assert list(rec["first_pkt"]) == [0, 3, 4, 5, 6, 7, 8, 9, 10]


def _parse(frame: bytes):
    ihl = 4 * (frame[0] & 0xF)
    bth = frame[ihl + 8: ihl + 20]
    return ihl, bth[0], (bth[1] >> 4) & 3, int.from_bytes(bth[9:12], "big"), bth


EXT_LEN = {0x06: 16, 0x0A: 16, 0x0B: 20, 0x09: 4, 0x03: 4, 0x05: 4, 0x16: 4, 0x17: 4,
           0x0D: 4, 0x0F: 4, 0x10: 4, 0x0C: 16, 0x13: 28, 0x14: 28, 0x11: 4, 0x12: 12}


@pytest.mark.parametrize("pmtu", (256, 1024, 4096))
def test_oracle_frames_are_wellformed_and_reassemble(pmtu):
    mr = np.random.default_rng(7).integers(0, 256, 5 * pmtu, dtype=np.uint8).tobytes()
    wrs = all_ops_cases(pmtu, len(mr), seed=pmtu)
    frames = SO.segment(mr, wrs, pmtu)
    i = 0
    for w in wrs:
        n = SO.packets_of(w, pmtu)
        data = b""
        for k in range(n):
            f = frames[i]
            i += 1
            assert O.verify_frame(f)
            assert O.inet_checksum(f[:20]) == 0  # IPv4 header checksum
            udp_len = len(f) - 20
            pseudo = f[12:20] + struct.pack("!BBH", 0, 17, udp_len)
            assert O.inet_checksum(pseudo + f[20:]) == 0  # UDP checksum over the final bytes
            ihl, opc, pad, psn, bth = _parse(f)
            assert psn == (w.psn + k) % (1 << 24)
            ext = EXT_LEN.get(opc, 0)
            payload = f[ihl + 20 + ext: len(f) - 4]
            assert payload[len(payload) - pad:] == b"\0" * pad
            data += payload[: len(payload) - pad]
            if w.op in SO.HEADER_ONLY:  # requests ask for an ACK, responses do not
                assert (bth[8] >> 7) == int(w.op <= SO.FETCH_ADD) and payload == b""
                continue
            assert (bth[8] >> 7) == (int(bool(w.flags & SO.SIGNALED)) if k == n - 1 and w.op != SO.READ_RESPONSE else 0)
        if w.op in SO.HEADER_ONLY:
            continue
        assert data == mr[w.mr_offset: w.mr_offset + w.length]
    assert i == len(frames)


def test_oracle_opcode_sequences():
    """FIRST/MIDDLE/LAST/ONLY per WR op (src/roce_sq.py:1259-1306, 1339-1395,
    src/roce_rq.py:399-431)."""
    mtu = 256

    def ops(op, length):
        w = SO.SegWR(op=op, mr_offset=0, length=length, psn=0, dqpn=1, src_ip=1, dst_ip=2, sport=3)
        return [b["opcode"] for b, _, _ in SO.wr_packets(w, mtu)]

    assert ops(SO.SEND, 0) == [0x04]
    assert ops(SO.SEND, 3 * mtu) == [0x00, 0x01, 0x02]
    assert ops(SO.SEND_WITH_IMM, 2 * mtu) == [0x00, 0x03]
    assert ops(SO.SEND_WITH_INV, 1) == [0x17]
    assert ops(SO.SEND_WITH_INV, mtu + 1) == [0x00, 0x16]
    assert ops(SO.RDMA_WRITE, mtu) == [0x0A]
    assert ops(SO.RDMA_WRITE, 3 * mtu) == [0x06, 0x07, 0x08]
    assert ops(SO.RDMA_WRITE_WITH_IMM, 0) == [0x0B]
    assert ops(SO.RDMA_WRITE_WITH_IMM, 2 * mtu + 1) == [0x06, 0x07, 0x09]
    assert ops(SO.READ_RESPONSE, 0) == [0x10]
    assert ops(SO.READ_RESPONSE, 4 * mtu) == [0x0D, 0x0E, 0x0E, 0x0F]
    assert ops(SO.READ_REQUEST, 4 * mtu) == [0x0C]
    assert ops(SO.COMPARE_SWAP, 0) == [0x13] and ops(SO.FETCH_ADD, 0) == [0x14]
    assert ops(SO.ACK, 0) == ops(SO.RNR_NAK, 0) == ops(SO.NAK, 0) == [0x11]
    assert ops(SO.ATOMIC_ACK, 0) == [0x12]


def test_oracle_header_only_fields():
    """The extension headers of the header-only packets, field by field
    (src/roce.py:263-297 layouts; values of src/roce_sq.py:1421-1463 and
    src/roce_rq.py:517-524, 767-853)."""
    base = dict(mr_offset=0, psn=(1 << 24) + 5, dqpn=0x123456, src_ip=1, dst_ip=2, sport=3,
                msn=0x1ABCDEF, remote_va=0x1122334455667788, rkey=0xCAFEBABE,
                swap=0x0102030405060708, comp=0xF0E0D0C0B0A09080, imm=0x47, length=12345)

    def pk(op):
        (bth, ext, sl), = SO.wr_packets(SO.SegWR(op=op, **base), 256)
        assert sl is None and bth["psn"] == 5 and bth["dqpn"] == 0x123456
        return bth, ext

    b, e = pk(SO.READ_REQUEST)
    assert b["ackreq"] == 1 and e == struct.pack("!QII", 0x1122334455667788, 0xCAFEBABE, 12345)
    for op, opc in ((SO.COMPARE_SWAP, 0x13), (SO.FETCH_ADD, 0x14)):
        b, e = pk(op)
        assert b["opcode"] == opc and b["ackreq"] == 1
        assert e == struct.pack("!QIQQ", 0x1122334455667788, 0xCAFEBABE, 0x0102030405060708,
                                0xF0E0D0C0B0A09080)
    # AETH byte 0 = code << 5 | value; msn masked to 24 bits
    assert pk(SO.ACK)[1] == bytes([0x1F]) + b"\xab\xcd\xef"
    assert pk(SO.RNR_NAK)[1] == bytes([0x20 | 0x07]) + b"\xab\xcd\xef"
    assert pk(SO.NAK)[1] == bytes([0x60 | 0x07]) + b"\xab\xcd\xef"
    b, e = pk(SO.ATOMIC_ACK)
    assert b.get("ackreq", 0) == 0
    assert e == bytes([0x1F]) + b"\xab\xcd\xef" + struct.pack("!Q", 0x0102030405060708)


def test_oracle_lengths_cover_boundaries():
    assert {SO.wr_pkt_num(n, 256) for n in lengths_for(256)} == {1, 2, 4}


def test_header_only_oracle_matches_packet_api_mirror():
    """The oracle's header-only frames equal the packet-object mirror's build of
    the reference's own constructor calls (ICRC field given explicitly, so no
    engine is needed): src/roce_sq.py:1421-1463, src/roce_rq.py:517-524,
    767-853."""
    from roce_icrc import roce as R

    va, rkey = 0x7F00AA5500001000, 0x1234ABCD
    common = dict(mr_offset=0, dqpn=0x2A, src_ip=0x0A010130, dst_ip=0x0A01010F, sport=0x11)
    cases = [
        (SO.SegWR(op=SO.READ_REQUEST, length=70000, psn=10, remote_va=va, rkey=rkey, **common),
         R.BTH(opcode=0x0C, psn=10, dqpn=0x2A, ackreq=True) / R.RETH(va=va, rkey=rkey, dlen=70000)),
        (SO.SegWR(op=SO.COMPARE_SWAP, length=0, psn=11, remote_va=va, rkey=rkey, swap=7, comp=9,
                  **common),
         R.BTH(opcode=0x13, psn=11, dqpn=0x2A, ackreq=True)
         / R.AtomicETH(va=va, rkey=rkey, comp=9, swap=7)),
        (SO.SegWR(op=SO.ACK, length=0, psn=13, msn=3, **common),
         R.BTH(opcode=0x11, psn=13, dqpn=0x2A) / R.AETH(code="ACK", value=31, msn=3)),
        (SO.SegWR(op=SO.RNR_NAK, length=0, psn=14, msn=4, imm=9, **common),
         R.BTH(opcode=0x11, psn=14, dqpn=0x2A) / R.AETH(code="RNR", value=9, msn=4)),
        (SO.SegWR(op=SO.NAK, length=0, psn=16, msn=6, imm=3, **common),
         R.BTH(opcode=0x11, psn=16, dqpn=0x2A) / R.AETH(code="NAK", value=3, msn=6)),
        (SO.SegWR(op=SO.ATOMIC_ACK, length=0, psn=17, msn=7, swap=0xDEADBEEF00C0FFEE, **common),
         R.BTH(opcode=0x12, psn=17, dqpn=0x2A) / R.AETH(code="ACK", value=31, msn=7)
         / R.AtomicAckETH(orig=0xDEADBEEF00C0FFEE)),
    ]
    for wr, pkt in cases:
        (want,) = SO.segment(b"", [wr], 256)
        pkt[R.BTH].icrc = int.from_bytes(want[-4:], "big")  # FCSField "!I": wire bytes as-is
        ip = R.l3_packet(pkt, dst="10.1.1.15", sport=0x11, src="10.1.1.48")
        got = bytes(ip)
        # the mirror leaves the UDP checksum to the emit path; compare all but it
        assert got[:26] == want[:26] and got[28:] == want[28:], wr.op

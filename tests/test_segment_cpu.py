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
    assert slot % 256 == 0 and slot >= 60 + pmtu + 4 and slot - (60 + pmtu + 4) < 256


def test_plan_rejects_bad_arguments():
    rec = E.seg_wrs(2)
    with pytest.raises(E.IcrcError):
        E.segment_plan(rec, 1000)  # not an IB MTU
    rec[1]["op"] = 6
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
    assert offs == dict(mr_offset=0, remote_va=8, length=16, psn=20, dqpn=24, src_ip=28,
                        dst_ip=32, rkey=36, imm=40, msn=44, sport=48, op=50, flags=51,
                        first_pkt=52, reserved=56)


def _parse(frame: bytes):
    ihl = 4 * (frame[0] & 0xF)
    bth = frame[ihl + 8: ihl + 20]
    return ihl, bth[0], (bth[1] >> 4) & 3, int.from_bytes(bth[9:12], "big"), bth


EXT_LEN = {0x06: 16, 0x0A: 16, 0x0B: 20, 0x09: 4, 0x03: 4, 0x05: 4, 0x16: 4, 0x17: 4,
           0x0D: 4, 0x0F: 4, 0x10: 4}


@pytest.mark.parametrize("pmtu", (256, 1024, 4096))
def test_oracle_frames_are_wellformed_and_reassemble(pmtu):
    mr = np.random.default_rng(7).integers(0, 256, 5 * pmtu, dtype=np.uint8).tobytes()
    wrs = all_ops_cases(pmtu, len(mr), seed=pmtu)
    frames = SO.segment(mr, wrs, pmtu)
    i = 0
    for w in wrs:
        n = SO.wr_pkt_num(w.length, pmtu)
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
            assert (bth[8] >> 7) == (int(bool(w.flags & SO.SIGNALED)) if k == n - 1 and w.op != SO.READ_RESPONSE else 0)
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


def test_oracle_lengths_cover_boundaries():
    assert {SO.wr_pkt_num(n, 256) for n in lengths_for(256)} == {1, 2, 4}

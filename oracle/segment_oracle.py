"""CPU oracle for MR -> packet segmentation (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product (``roce-sim_amd/``) never does: its
segmentation runs in the HIP kernel behind ``ricrc_segment[_dev]``.

What it restates (datenlord/roce-sim, read as text; the reference cannot be
imported here because scapy is absent):

* ``Util.compute_wr_pkt_num``  ``src/roce_util.py:183-185``:
  ``ceil(size / mtu) if size > 0 else 1``.
* ``TXLogic.process_send_req`` ``src/roce_sq.py:1243-1321``: SEND_FIRST,
  SEND_MIDDLE x (n - 2), then SEND_LAST[_WITH_IMMEDIATE|_WITH_INVALIDATE] or,
  for one packet, SEND_ONLY[...]; ImmDt / IETH on the last packet only;
  ackreq and solicited from the WR flags on the last packet only; the last
  packet carries ``data[(n-1)*mtu : size]`` only when ``size > 0``.
* ``TXLogic.process_write_req`` ``src/roce_sq.py:1323-1411``: RETH(va, rkey,
  dlen = size) on RDMA_WRITE_FIRST and RDMA_WRITE_ONLY, ImmDt on
  RDMA_WRITE_LAST_WITH_IMMEDIATE, RETHImmDt on RDMA_WRITE_ONLY_WITH_IMMEDIATE;
  solicited only for the WITH_IMM last/only packet.
* ``ReadReqCtx.commit`` ``src/roce_rq.py:388-438``: AETH(code ACK, value
  CREDIT_CNT_INVALID = 31, msn) on READ_RESPONSE_FIRST / LAST / ONLY, none on
  MIDDLE; ackreq and solicited 0.
* The IP/UDP wrap of ``TXLogic.send_ip_pkt`` ``src/roce_sq.py:1186-1197`` and
  ``RXLogic.send_pkt`` ``src/roce_rq.py:705-731`` (UDP sport = own QPN,
  dport 4791), padding per ``src/roce_util.py:187-199`` and the scapy
  serialisation, both through ``icrc_oracle.build_frame``.
* PSN of packet k: ``cpsn + k``, a 24-bit BTH field (scapy masks it), i.e.
  ``(cpsn + k) mod 2^24``.
* Header-only packets, one per WR, no payload:
  ``TXLogic.process_read_req`` ``src/roce_sq.py:1413-1439`` -- BTH(
  RDMA_READ_REQUEST, psn, dqpn, ackreq=True) / RETH(va, rkey, dlen=size);
  ``TXLogic.process_atomic_req`` ``src/roce_sq.py:1441-1466`` -- BTH(
  COMPARE_SWAP | FETCH_ADD, ackreq=True) / AtomicETH(va, rkey, comp, swap);
  ``RXLogic.process_ack`` ``src/roce_rq.py:767-776`` -- BTH(ACKNOWLEDGE) /
  AETH(code ACK, value CREDIT_CNT_INVALID, msn); ``process_nak_rnr``
  ``:778-788`` -- AETH(code RNR, value = min_rnr_timer, msn);
  ``process_nak_seq_err`` ``:805-814`` -- AETH(code NAK, value 0, msn);
  ``process_nak_err`` ``:827-853`` -- AETH(code NAK, value 1 / 2 / 3, msn);
  ``AtomicReqCtx.commit`` ``src/roce_rq.py:517-525`` -- BTH(
  ATOMIC_ACKNOWLEDGE) / AETH(ACK, CREDIT_CNT_INVALID, msn) /
  AtomicAckETH(orig).  The AETH value is a 5-bit field, the msn 24 bits.

Parity status: **parity unpinned** for the segmentation rules (no reference
test holds segmented frames; restated from the file:line ranges above).  The
frame bytes go through ``build_frame``, whose serialisation reproduces the
SURVEY Appendix B example byte for byte, and the ICRC is ``zlib.crc32``.
"""
from __future__ import annotations

import math
import os
import sys
from dataclasses import dataclass

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import icrc_oracle as O  # noqa: E402

# WR operations (include/roce_icrc.h RICRC_SEG_*)
SEND, SEND_WITH_IMM, SEND_WITH_INV, RDMA_WRITE, RDMA_WRITE_WITH_IMM, READ_RESPONSE = range(6)
READ_REQUEST, COMPARE_SWAP, FETCH_ADD, ACK, RNR_NAK, NAK, ATOMIC_ACK = range(6, 13)
HEADER_ONLY = (READ_REQUEST, COMPARE_SWAP, FETCH_ADD, ACK, RNR_NAK, NAK, ATOMIC_ACK)
AETH_ACK, AETH_RNR, AETH_NAK = 0, 1, 3  # AETH.code, src/roce.py:267
SIGNALED, SOLICITED = 1, 2
CREDIT_CNT_INVALID = 31  # src/roce_enum.py:8
MAX_PSN = 1 << 24  # src/roce_enum.py:19

# RC opcodes (src/roce.py opcode table; src/roce_enum.py:282-304)
OP = dict(
    SEND_FIRST=0x00, SEND_MIDDLE=0x01, SEND_LAST=0x02, SEND_LAST_WITH_IMMEDIATE=0x03,
    SEND_ONLY=0x04, SEND_ONLY_WITH_IMMEDIATE=0x05, RDMA_WRITE_FIRST=0x06,
    RDMA_WRITE_MIDDLE=0x07, RDMA_WRITE_LAST=0x08, RDMA_WRITE_LAST_WITH_IMMEDIATE=0x09,
    RDMA_WRITE_ONLY=0x0A, RDMA_WRITE_ONLY_WITH_IMMEDIATE=0x0B,
    RDMA_READ_RESPONSE_FIRST=0x0D, RDMA_READ_RESPONSE_MIDDLE=0x0E,
    RDMA_READ_RESPONSE_LAST=0x0F, RDMA_READ_RESPONSE_ONLY=0x10,
    SEND_LAST_WITH_INVALIDATE=0x16, SEND_ONLY_WITH_INVALIDATE=0x17,
    RDMA_READ_REQUEST=0x0C, ACKNOWLEDGE=0x11, ATOMIC_ACKNOWLEDGE=0x12, COMPARE_SWAP=0x13,
    FETCH_ADD=0x14,
)


@dataclass
class SegWR:
    """One work request (the fields of ``ricrc_seg_wr``)."""

    op: int
    mr_offset: int
    length: int
    psn: int
    dqpn: int
    src_ip: int
    dst_ip: int
    sport: int
    flags: int = 0
    imm: int = 0
    remote_va: int = 0
    rkey: int = 0
    msn: int = 0
    swap: int = 0  # AtomicETH.swap; AtomicAckETH.orig for ATOMIC_ACK
    comp: int = 0  # AtomicETH.comp


def wr_pkt_num(size: int, mtu: int) -> int:
    """Util.compute_wr_pkt_num, src/roce_util.py:183-185."""
    return math.ceil(size / mtu) if size > 0 else 1


def packets_of(wr: SegWR, mtu: int) -> int:
    """Packets one WR emits: compute_wr_pkt_num for the payload ops, 1 for the
    header-only ones (a read request asks for its response packets but is one
    packet itself, src/roce_sq.py:1413-1439)."""
    return 1 if wr.op in HEADER_ONLY else wr_pkt_num(wr.length, mtu)


def _ip(a: int) -> str:
    return ".".join(str((a >> s) & 0xFF) for s in (24, 16, 8, 0))


def wr_packets(wr: SegWR, mtu: int):
    """The (bth fields, ext bytes, payload or None) of every packet of one WR,
    in emit order -- the opcode / extension-header / slicing rules of
    src/roce_sq.py:1243-1411 and src/roce_rq.py:388-438."""
    n = wr_pkt_num(wr.length, mtu)
    sig = bool(wr.flags & SIGNALED)
    sol = bool(wr.flags & SOLICITED)
    out = []

    def psn(k):
        return (wr.psn + k) % MAX_PSN

    def mid_slice(k):
        return (k * mtu, (k + 1) * mtu)

    last_slice = ((n - 1) * mtu, wr.length) if wr.length > 0 else None
    if wr.op in (SEND, SEND_WITH_IMM, SEND_WITH_INV):
        for k in range(n - 1):  # src/roce_sq.py:1259-1283
            opc = OP["SEND_FIRST"] if k == 0 else OP["SEND_MIDDLE"]
            out.append((dict(opcode=opc, psn=psn(k), dqpn=wr.dqpn), b"", mid_slice(k)))
        kind = {SEND: "", SEND_WITH_IMM: "_WITH_IMMEDIATE", SEND_WITH_INV: "_WITH_INVALIDATE"}[wr.op]
        opc = OP[("SEND_ONLY" if n == 1 else "SEND_LAST") + kind]
        ext = b""
        if wr.op == SEND_WITH_IMM:
            ext = O.immdt_bytes(wr.imm)
        elif wr.op == SEND_WITH_INV:
            ext = O.ieth_bytes(wr.imm)
        bth = dict(opcode=opc, psn=psn(n - 1), dqpn=wr.dqpn, ackreq=int(sig), solicited=int(sol))
        out.append((bth, ext, last_slice))
    elif wr.op in (RDMA_WRITE, RDMA_WRITE_WITH_IMM):
        reth = O.reth_bytes(wr.remote_va, wr.rkey, wr.length)
        for k in range(n - 1):  # src/roce_sq.py:1339-1365
            opc = OP["RDMA_WRITE_FIRST"] if k == 0 else OP["RDMA_WRITE_MIDDLE"]
            out.append((dict(opcode=opc, psn=psn(k), dqpn=wr.dqpn), reth if k == 0 else b"",
                        mid_slice(k)))
        imm = wr.op == RDMA_WRITE_WITH_IMM
        solicited = int(sol) if imm else 0
        if n == 1:
            if imm:
                opc = OP["RDMA_WRITE_ONLY_WITH_IMMEDIATE"]
                ext = O.reth_immdt_bytes(wr.remote_va, wr.rkey, wr.length, wr.imm)
            else:
                opc, ext = OP["RDMA_WRITE_ONLY"], reth
        else:
            if imm:
                opc, ext = OP["RDMA_WRITE_LAST_WITH_IMMEDIATE"], O.immdt_bytes(wr.imm)
            else:
                opc, ext = OP["RDMA_WRITE_LAST"], b""
        bth = dict(opcode=opc, psn=psn(n - 1), dqpn=wr.dqpn, ackreq=int(sig), solicited=solicited)
        out.append((bth, ext, last_slice))
    elif wr.op == READ_REQUEST:  # src/roce_sq.py:1421-1428
        bth = dict(opcode=OP["RDMA_READ_REQUEST"], psn=psn(0), dqpn=wr.dqpn, ackreq=1)
        out.append((bth, O.reth_bytes(wr.remote_va, wr.rkey, wr.length), None))
    elif wr.op in (COMPARE_SWAP, FETCH_ADD):  # src/roce_sq.py:1444-1463
        opc = OP["COMPARE_SWAP" if wr.op == COMPARE_SWAP else "FETCH_ADD"]
        bth = dict(opcode=opc, psn=psn(0), dqpn=wr.dqpn, ackreq=1)
        out.append((bth, O.atomic_eth_bytes(wr.remote_va, wr.rkey, wr.swap, wr.comp), None))
    elif wr.op in (ACK, RNR_NAK, NAK):  # src/roce_rq.py:767-853
        code = {ACK: AETH_ACK, RNR_NAK: AETH_RNR, NAK: AETH_NAK}[wr.op]
        value = CREDIT_CNT_INVALID if wr.op == ACK else wr.imm & 0x1F
        bth = dict(opcode=OP["ACKNOWLEDGE"], psn=psn(0), dqpn=wr.dqpn)
        out.append((bth, O.aeth_bytes(code=code, value=value, msn=wr.msn & 0xFFFFFF), None))
    elif wr.op == ATOMIC_ACK:  # src/roce_rq.py:517-525
        bth = dict(opcode=OP["ATOMIC_ACKNOWLEDGE"], psn=psn(0), dqpn=wr.dqpn)
        ext = O.aeth_bytes(code=AETH_ACK, value=CREDIT_CNT_INVALID, msn=wr.msn & 0xFFFFFF) + \
            O.atomic_ack_eth_bytes(wr.swap)
        out.append((bth, ext, None))
    elif wr.op == READ_RESPONSE:
        aeth = O.aeth_bytes(code=0, value=CREDIT_CNT_INVALID, msn=wr.msn)
        for k in range(n - 1):  # src/roce_rq.py:399-421
            opc = OP["RDMA_READ_RESPONSE_FIRST"] if k == 0 else OP["RDMA_READ_RESPONSE_MIDDLE"]
            out.append((dict(opcode=opc, psn=psn(k), dqpn=wr.dqpn), aeth if k == 0 else b"",
                        mid_slice(k)))
        opc = OP["RDMA_READ_RESPONSE_ONLY" if n == 1 else "RDMA_READ_RESPONSE_LAST"]
        out.append((dict(opcode=opc, psn=psn(n - 1), dqpn=wr.dqpn), aeth, last_slice))
    else:
        raise ValueError(f"unknown WR op {wr.op}")
    return out


def segment(mr: bytes, wrs: list[SegWR], mtu: int) -> list[bytes]:
    """Every wire frame the WRs produce, in order (WR by WR, packet by packet)."""
    frames = []
    for wr in wrs:
        for bth, ext, sl in wr_packets(wr, mtu):
            payload = None if sl is None else bytes(mr[wr.mr_offset + sl[0]: wr.mr_offset + sl[1]])
            frames.append(O.build_frame(_ip(wr.src_ip), _ip(wr.dst_ip), wr.sport, bth, ext, payload))
    return frames

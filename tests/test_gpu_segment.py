"""GPU parity of the MR -> packet segmentation kernel (ricrc_segment[_dev])
against the segmentation oracle (oracle/segment_oracle.py): bit-exact frame
bytes, lengths and ICRCs for every WR op, boundary lengths, PMTUs, lane
settings and unaligned MR offsets; invalid WRs; full-size batches through
size-independent properties (ICRC verify, payload reassembly, checksums)."""
from __future__ import annotations

import struct

import numpy as np
import pytest

import icrc_oracle as O
import segment_oracle as SO
from roce_icrc import engine as E
from segment_cases import DST_IP, SRC_IP, all_ops_cases, to_records

pytestmark = pytest.mark.gpu


def _check_against_oracle(eng, mr: bytes, wrs, pmtu, lanes=0):
    rec = to_records(wrs)
    frames, lens, icrc, st = eng.segment(mr, rec, pmtu)
    want = SO.segment(mr, wrs, pmtu)
    assert len(want) == frames.shape[0]
    assert not st.any()
    for p, f in enumerate(want):
        assert lens[p] == len(f), p
        got = frames[p, : len(f)].tobytes()
        if got != f:
            diff = [i for i in range(len(f)) if got[i] != f[i]]
            raise AssertionError(f"packet {p}: {len(diff)} bytes differ, first at {diff[:8]}")
        assert icrc[p] == O.icrc_of_frame(f)
        # slot bytes up to the end of the frame's last 16 * lanes-byte run are
        # zero (include/roce_icrc.h; the next 16-byte boundary at least)
        run = 16 * (lanes or 1)
        tail = min((-len(f)) % run, frames.shape[1] - len(f))
        assert not frames[p, len(f): len(f) + tail].any()


@pytest.mark.parametrize("pmtu", (256, 1024, 4096))
@pytest.mark.parametrize("lanes", (0, 2, 4, 8, 16))
def test_every_op_and_boundary_length(engine, pmtu, lanes):
    mr = np.random.default_rng(pmtu + lanes).integers(0, 256, 5 * pmtu + 7, dtype=np.uint8).tobytes()
    wrs = all_ops_cases(pmtu, len(mr), seed=pmtu * 7 + lanes)
    engine.set_lanes(lanes)
    try:
        _check_against_oracle(engine, mr, wrs, pmtu, lanes)
    finally:
        engine.set_lanes(0)


@pytest.mark.parametrize("misalign", range(8))
def test_unaligned_mr_offsets(engine, misalign):
    pmtu = 1024
    mr = np.random.default_rng(misalign).integers(0, 256, 8 * pmtu, dtype=np.uint8).tobytes()
    wrs = [SO.SegWR(op=op, mr_offset=16 * i + misalign, length=ln, psn=i, dqpn=0x11,
                    src_ip=SRC_IP, dst_ip=DST_IP, sport=2, flags=SO.SIGNALED)
           for i, (op, ln) in enumerate([(0, 3 * pmtu + 5), (3, 2 * pmtu - 3), (5, 4097), (1, 13)])]
    _check_against_oracle(engine, mr, wrs, pmtu)


def test_message_ending_at_mr_end(engine):
    """The last chunk of a message that ends the MR is read byte by byte
    (no 16-byte over-read past the MR)."""
    pmtu = 256
    for tail in range(1, 17):
        mr = bytes(range(256)) * 3 + bytes(tail)
        n = 2 * pmtu + tail - 3
        wrs = [SO.SegWR(op=SO.SEND, mr_offset=len(mr) - n, length=n, psn=5, dqpn=3,
                        src_ip=SRC_IP, dst_ip=DST_IP, sport=9)]
        _check_against_oracle(engine, mr, wrs, pmtu)


def test_psn_wraps_at_2_pow_24(engine):
    pmtu = 256
    mr = bytes(4 * pmtu)
    wrs = [SO.SegWR(op=SO.RDMA_WRITE, mr_offset=0, length=4 * pmtu, psn=(1 << 24) - 2, dqpn=1,
                    src_ip=SRC_IP, dst_ip=DST_IP, sport=1)]
    _check_against_oracle(engine, mr, wrs, pmtu)


def test_sim_send_success_config1(engine):
    """Config 1: a 1-byte SEND_ONLY, signaled, from the MR."""
    wr = SO.SegWR(op=SO.SEND, mr_offset=0, length=1, psn=0, dqpn=0x11, src_ip=SRC_IP,
                  dst_ip=DST_IP, sport=2, flags=SO.SIGNALED)
    frames, lens, icrc, st = engine.segment(b"\xff", to_records([wr]), 1024)
    assert frames[0, : lens[0]].tobytes() == O.sim_send_success_frame()
    assert icrc[0] == 0x1BE21D75


def test_host_call_rejects_out_of_range_wr(engine):
    rec = to_records([SO.SegWR(op=0, mr_offset=10, length=100, psn=0, dqpn=0, src_ip=0,
                               dst_ip=0, sport=0)])
    with pytest.raises(E.IcrcError):
        engine.segment(bytes(64), rec, 256)


def test_device_call_flags_bad_wrs(engine):
    """Device-resident WRs are validated in the kernel: out-of-range MR, bad
    op -> len 0, status SEG_BAD; the good WR is still built."""
    import torch

    pmtu = 256
    mr = np.random.default_rng(3).integers(0, 256, 2048, dtype=np.uint8)
    wrs = [SO.SegWR(op=0, mr_offset=100, length=600, psn=7, dqpn=1, src_ip=SRC_IP,
                    dst_ip=DST_IP, sport=4),
           SO.SegWR(op=3, mr_offset=2000, length=100, psn=0, dqpn=1, src_ip=SRC_IP,
                    dst_ip=DST_IP, sport=4)]
    rec = to_records(wrs)
    npkts, slot = E.segment_plan(rec, pmtu)
    rec2 = np.concatenate([rec, to_records([wrs[0]])])
    rec2[2]["first_pkt"] = npkts
    rec2[2]["op"] = E.SEG_NUM_OPS
    npkts += 1
    dev = torch.device("cuda", 0)
    d_mr = torch.from_numpy(mr).to(dev)
    d_wrs = torch.from_numpy(rec2.view(np.uint8)).to(dev)
    d_frames = torch.zeros(npkts * slot, dtype=torch.uint8, device=dev)
    d_lens = torch.zeros(npkts, dtype=torch.int32, device=dev)
    d_icrc = torch.zeros(npkts, dtype=torch.int32, device=dev)
    d_st = torch.zeros(npkts, dtype=torch.uint8, device=dev)
    engine.segment_dev(d_mr, mr.size, d_wrs, 3, pmtu, npkts, d_frames, slot, d_lens, d_icrc, d_st)
    torch.cuda.synchronize()
    lens = d_lens.cpu().numpy().view(np.uint32)
    st = d_st.cpu().numpy()
    want = SO.segment(mr.tobytes(), wrs[:1], pmtu)
    assert list(lens[: len(want)]) == [len(f) for f in want]
    fr = d_frames.cpu().numpy().reshape(npkts, slot)
    for p, f in enumerate(want):
        assert fr[p, : len(f)].tobytes() == f
    assert (st[: len(want)] == 0).all()
    assert (lens[len(want):] == 0).all() and (st[len(want):] == E.PKT_SEG_BAD).all()


def test_matches_packet_api_emit(engine):
    """The kernel's frames equal what the packet-object mirror of roce-sim
    builds for the same requests (roce_icrc.roce: BTH/RETH/ImmDt/... / Raw,
    l3_packet, emit_batch)."""
    from roce_icrc import roce as R

    pmtu = 256
    mr = bytes((i * 37 + 11) & 0xFF for i in range(3 * pmtu))
    wrs = [SO.SegWR(op=SO.RDMA_WRITE_WITH_IMM, mr_offset=5, length=2 * pmtu + 9, psn=100,
                    dqpn=0x33, src_ip=SRC_IP, dst_ip=DST_IP, sport=7, flags=3, imm=0xABCD,
                    remote_va=0x1000, rkey=0x55),
           SO.SegWR(op=SO.READ_RESPONSE, mr_offset=0, length=pmtu + 2, psn=9, dqpn=0x34,
                    src_ip=SRC_IP, dst_ip=DST_IP, sport=8, msn=77)]
    frames, lens, _, _ = engine.segment(mr, to_records(wrs), pmtu)
    reth = R.RETH(va=0x1000, rkey=0x55, dlen=2 * pmtu + 9)
    aeth = R.AETH(code=0, value=31, msn=77)
    pkts = [
        R.l3_packet(R.BTH(opcode=0x06, psn=100, dqpn=0x33) / reth / R.Raw(load=mr[5:5 + pmtu]),
                    dst="10.1.1.15", sport=7, src="10.1.1.48"),
        R.l3_packet(R.BTH(opcode=0x07, psn=101, dqpn=0x33) / R.Raw(load=mr[5 + pmtu:5 + 2 * pmtu]),
                    dst="10.1.1.15", sport=7, src="10.1.1.48"),
        R.l3_packet(R.BTH(opcode=0x09, psn=102, dqpn=0x33, ackreq=1, solicited=1)
                    / R.ImmDt(data=0xABCD) / R.Raw(load=mr[5 + 2 * pmtu:5 + 2 * pmtu + 9]),
                    dst="10.1.1.15", sport=7, src="10.1.1.48"),
        R.l3_packet(R.BTH(opcode=0x0D, psn=9, dqpn=0x34) / aeth / R.Raw(load=mr[0:pmtu]),
                    dst="10.1.1.15", sport=8, src="10.1.1.48"),
        R.l3_packet(R.BTH(opcode=0x0F, psn=10, dqpn=0x34) / R.AETH(code=0, value=31, msn=77)
                    / R.Raw(load=mr[pmtu:pmtu + 2]), dst="10.1.1.15", sport=8, src="10.1.1.48"),
    ]
    emitted = R.emit_batch(pkts)
    assert len(emitted) == frames.shape[0]
    for p, f in enumerate(emitted):
        assert frames[p, : lens[p]].tobytes() == bytes(f), p


def test_full_size_batch_properties(engine):
    """A bench-sized batch (2^18 packets of 4 KiB PMTU): every frame verifies,
    payloads reassemble to the MR, IPv4/UDP checksums hold (sampled), and a
    strided sample is bit-exact against the oracle."""
    import torch

    pmtu, msg = 4096, 64 * 4096 + 1000  # 65 packets per WR, ragged last packet
    nwr = 4096
    rng = np.random.default_rng(11)
    mr = rng.integers(0, 256, nwr * msg + 3, dtype=np.uint8)
    rec = E.seg_wrs(nwr)
    rec["op"] = rng.integers(0, 6, nwr)
    rec["mr_offset"] = np.arange(nwr, dtype=np.uint64) * msg + 3
    rec["length"] = msg
    rec["psn"] = rng.integers(0, 1 << 24, nwr)
    rec["dqpn"] = rng.integers(0, 1 << 24, nwr)
    rec["src_ip"], rec["dst_ip"] = SRC_IP, DST_IP
    rec["sport"] = rng.integers(0, 1 << 16, nwr)
    rec["flags"] = rng.integers(0, 4, nwr)
    rec["imm"] = rng.integers(0, 1 << 32, nwr, dtype=np.uint64)
    npkts, slot = E.segment_plan(rec, pmtu)
    dev = torch.device("cuda", 0)
    d_mr = torch.from_numpy(mr).to(dev)
    d_wrs = torch.from_numpy(rec.view(np.uint8)).to(dev)
    d_frames = torch.empty(npkts * slot, dtype=torch.uint8, device=dev)
    d_lens = torch.empty(npkts, dtype=torch.int32, device=dev)
    d_icrc = torch.empty(npkts, dtype=torch.int32, device=dev)
    d_st = torch.empty(npkts, dtype=torch.uint8, device=dev)
    engine.segment_dev(d_mr, mr.size, d_wrs, nwr, pmtu, npkts, d_frames, slot, d_lens, d_icrc, d_st)
    # verify every frame's ICRC with the verify kernel
    d_offs = torch.arange(npkts, dtype=torch.int64, device=dev) * slot
    d_ok = torch.empty(npkts, dtype=torch.uint8, device=dev)
    engine.verify_batch_dev(d_frames, d_offs, d_lens, npkts, d_ok)
    torch.cuda.synchronize()
    assert int(d_st.sum()) == 0
    assert bool((d_ok == 1).all())
    lens = d_lens.cpu().numpy().view(np.uint32)
    frames = d_frames.cpu().numpy().reshape(npkts, slot)
    icrc = d_icrc.cpu().numpy().view(np.uint32)
    # payload reassembly: full middle packets carry MR bytes at a fixed offset
    per = npkts // nwr
    mids = frames.reshape(nwr, per, slot)[:, 1:-1]
    hdr = 40  # middle packets of every op have no extension header
    want = mr[3: 3 + nwr * msg].reshape(nwr, msg)[:, pmtu: (per - 1) * pmtu].reshape(nwr, per - 2, pmtu)
    assert np.array_equal(mids[:, :, hdr: hdr + pmtu], want)
    # sampled exact parity against the oracle (a few WRs, every packet)
    wr_objs = []
    for w in (0, 1, 2, 3, 4, 5, 777, nwr - 1):
        r = rec[w]
        wr_objs.append((w, SO.SegWR(op=int(r["op"]), mr_offset=int(r["mr_offset"]),
                                    length=int(r["length"]), psn=int(r["psn"]),
                                    dqpn=int(r["dqpn"]), src_ip=SRC_IP, dst_ip=DST_IP,
                                    sport=int(r["sport"]), flags=int(r["flags"]),
                                    imm=int(r["imm"]))))
    for w, wo in wr_objs:
        sub = SO.segment(memoryview(mr)[: int(wo.mr_offset) + wo.length], [wo], pmtu)
        for k, f in enumerate(sub):
            p = w * per + k
            assert lens[p] == len(f)
            assert frames[p, : len(f)].tobytes() == f
            assert icrc[p] == O.icrc_of_frame(f)
    # checksums on a sample of frames
    for p in range(0, npkts, 997):
        f = frames[p, : lens[p]].tobytes()
        assert O.inet_checksum(f[:20]) == 0
        pseudo = f[12:20] + struct.pack("!BBH", 0, 17, len(f) - 20)
        assert O.inet_checksum(pseudo + f[20:]) == 0


def test_mr_offsets_beyond_4_gib(engine):
    """A 4 GiB + 1 MiB device MR: WRs that straddle 2^32, start above it and
    end exactly at the MR end are segmented bit-exactly (64-bit MR offsets;
    the MR-end guard above 2^32).  The oracle sees the same bytes rebased to
    a small host array (frames carry no MR offset)."""
    import torch

    pmtu = 1024
    mr_bytes = (1 << 32) + (1 << 20)
    base = (1 << 32) - 8192
    tail = np.random.default_rng(99).integers(0, 256, mr_bytes - base, dtype=np.uint8)
    spans = [((1 << 32) - 3001, 9000, SO.SEND), ((1 << 32) + 77, 3 * pmtu + 5, SO.RDMA_WRITE),
             (mr_bytes - (2 * pmtu + 13), 2 * pmtu + 13, SO.READ_RESPONSE)]
    wrs = [SO.SegWR(op=op, mr_offset=off, length=ln, psn=100 * i, dqpn=0x21, src_ip=SRC_IP,
                    dst_ip=DST_IP, sport=5, flags=SO.SIGNALED)
           for i, (off, ln, op) in enumerate(spans)]
    rebased = [SO.SegWR(op=w.op, mr_offset=w.mr_offset - base, length=w.length, psn=w.psn,
                        dqpn=w.dqpn, src_ip=w.src_ip, dst_ip=w.dst_ip, sport=w.sport,
                        flags=w.flags) for w in wrs]
    want = SO.segment(tail.tobytes(), rebased, pmtu)
    rec = to_records(wrs)
    npkts, slot = E.segment_plan(rec, pmtu)
    assert npkts == len(want)
    dev = torch.device("cuda", 0)
    d_mr = torch.empty(mr_bytes, dtype=torch.uint8, device=dev)
    d_mr[base:].copy_(torch.from_numpy(tail))
    d_wrs = torch.from_numpy(rec.view(np.uint8)).to(dev)
    d_frames = torch.zeros(npkts * slot, dtype=torch.uint8, device=dev)
    d_lens = torch.zeros(npkts, dtype=torch.int32, device=dev)
    d_icrc = torch.zeros(npkts, dtype=torch.int32, device=dev)
    d_st = torch.zeros(npkts, dtype=torch.uint8, device=dev)
    engine.segment_dev(d_mr, mr_bytes, d_wrs, len(wrs), pmtu, npkts, d_frames, slot, d_lens,
                       d_icrc, d_st)
    torch.cuda.synchronize()
    lens = d_lens.cpu().numpy().view(np.uint32)
    icrc = d_icrc.cpu().numpy().view(np.uint32)
    fr = d_frames.cpu().numpy().reshape(npkts, slot)
    assert not d_st.cpu().numpy().any()
    for p, f in enumerate(want):
        assert lens[p] == len(f), p
        assert fr[p, : len(f)].tobytes() == f, p
        assert icrc[p] == O.icrc_of_frame(f), p
    del d_mr
    torch.cuda.empty_cache()


def test_header_only_ops_match_packet_api(engine):
    """Read request, CompareSwap / FetchAdd, ACK, RNR NAK, sequence and error
    NAKs and the atomic acknowledge built by the kernel equal what the
    packet-object mirror builds for the reference's own calls
    (src/roce_sq.py:1421-1463, src/roce_rq.py:517-524, 767-853)."""
    from roce_icrc import roce as R

    va, rkey, swap, comp = 0x7F00AA5500001000, 0x1234ABCD, 0x0102030405060708, 0xFFEEDDCCBBAA9988
    common = dict(mr_offset=0, dqpn=0x2A, src_ip=SRC_IP, dst_ip=DST_IP, sport=0x11)
    wrs = [SO.SegWR(op=SO.READ_REQUEST, length=70000, psn=10, remote_va=va, rkey=rkey, **common),
           SO.SegWR(op=SO.COMPARE_SWAP, length=0, psn=11, remote_va=va, rkey=rkey, swap=swap,
                    comp=comp, **common),
           SO.SegWR(op=SO.FETCH_ADD, length=0, psn=12, remote_va=va + 8, rkey=rkey, swap=0,
                    comp=5, **common),
           SO.SegWR(op=SO.ACK, length=0, psn=13, msn=3, **common),
           SO.SegWR(op=SO.RNR_NAK, length=0, psn=14, msn=4, imm=9, **common),
           SO.SegWR(op=SO.NAK, length=0, psn=15, msn=5, imm=0, **common),
           SO.SegWR(op=SO.NAK, length=0, psn=16, msn=6, imm=2, **common),
           SO.SegWR(op=SO.ATOMIC_ACK, length=0, psn=17, msn=7, swap=0xDEADBEEF00C0FFEE, **common)]
    frames, lens, icrc, st = engine.segment(b"", to_records(wrs), 1024)
    assert not st.any() and frames.shape[0] == len(wrs)

    def wrap(p):
        return R.l3_packet(p, dst="10.1.1.15", sport=0x11, src="10.1.1.48")
    pkts = [
        wrap(R.BTH(opcode=0x0C, psn=10, dqpn=0x2A, ackreq=True) / R.RETH(va=va, rkey=rkey,
                                                                         dlen=70000)),
        wrap(R.BTH(opcode=0x13, psn=11, dqpn=0x2A, ackreq=True)
             / R.AtomicETH(va=va, rkey=rkey, comp=comp, swap=swap)),
        wrap(R.BTH(opcode=0x14, psn=12, dqpn=0x2A, ackreq=True)
             / R.AtomicETH(va=va + 8, rkey=rkey, comp=5, swap=0)),
        wrap(R.BTH(opcode=0x11, psn=13, dqpn=0x2A) / R.AETH(code="ACK", value=31, msn=3)),
        wrap(R.BTH(opcode=0x11, psn=14, dqpn=0x2A) / R.AETH(code="RNR", value=9, msn=4)),
        wrap(R.BTH(opcode=0x11, psn=15, dqpn=0x2A) / R.AETH(code="NAK", value=0, msn=5)),
        wrap(R.BTH(opcode=0x11, psn=16, dqpn=0x2A) / R.AETH(code="NAK", value=2, msn=6)),
        wrap(R.BTH(opcode=0x12, psn=17, dqpn=0x2A) / R.AETH(code="ACK", value=31, msn=7)
             / R.AtomicAckETH(orig=0xDEADBEEF00C0FFEE)),
    ]
    emitted = R.emit_batch(pkts)
    want = SO.segment(b"", wrs, 1024)
    for p, f in enumerate(emitted):
        assert bytes(f) == want[p], p
        assert frames[p, : lens[p]].tobytes() == bytes(f), p
        assert icrc[p] == O.icrc_of_frame(f)


@pytest.mark.parametrize("lanes", (0, 2, 16))
def test_mixed_burst_is_one_launch_without_an_mr(engine, lanes):
    """A responder-style burst -- read responses, ACKs, NAKs, atomic acks --
    interleaved with requester packets in ONE ricrc_segment_dev call (one
    segmentation launch); then a header-only burst with no MR at all (d_mr
    NULL, mr_bytes 0).  Bit-exact against the oracle."""
    import torch

    pmtu = 256
    rng = np.random.default_rng(21 + lanes)
    mr = rng.integers(0, 256, 8 * pmtu + 3, dtype=np.uint8)
    wrs = []
    for i in range(300):
        op = int(rng.integers(0, SO.ATOMIC_ACK + 1))
        length = int(rng.integers(0, 3 * pmtu)) if op < SO.READ_REQUEST else int(rng.integers(0, 1 << 20))
        off = int(rng.integers(0, mr.size - length + 1)) if op < SO.READ_REQUEST else 0
        wrs.append(SO.SegWR(op=op, mr_offset=off, length=length, psn=int(rng.integers(0, 1 << 24)),
                            dqpn=int(rng.integers(0, 1 << 24)), src_ip=SRC_IP, dst_ip=DST_IP,
                            sport=int(rng.integers(0, 1 << 16)), flags=int(rng.integers(0, 4)),
                            imm=int(rng.integers(0, 1 << 32)), remote_va=int(rng.integers(0, 1 << 63)),
                            rkey=int(rng.integers(0, 1 << 32)), msn=int(rng.integers(0, 1 << 24)),
                            swap=int(rng.integers(0, 1 << 63)), comp=int(rng.integers(0, 1 << 63))))
    dev = torch.device("cuda", 0)
    engine.set_lanes(lanes)
    try:
        for batch, use_mr in ((wrs, True), ([w for w in wrs if w.op in SO.HEADER_ONLY], False)):
            rec = to_records(batch)
            npkts, slot = E.segment_plan(rec, pmtu)
            want = SO.segment(mr.tobytes(), batch, pmtu)
            assert npkts == len(want)
            d_mr = torch.from_numpy(mr).to(dev) if use_mr else None
            d_wrs = torch.from_numpy(rec.view(np.uint8)).to(dev)
            d_frames = torch.zeros(npkts * slot, dtype=torch.uint8, device=dev)
            d_lens = torch.zeros(npkts, dtype=torch.int32, device=dev)
            d_icrc = torch.zeros(npkts, dtype=torch.int32, device=dev)
            d_st = torch.full((npkts,), 0xFF, dtype=torch.uint8, device=dev)
            engine.segment_dev(d_mr, mr.size if use_mr else 0, d_wrs, len(batch), pmtu, npkts,
                               d_frames, slot, d_lens, d_icrc, d_st)
            torch.cuda.synchronize()
            lens = d_lens.cpu().numpy().view(np.uint32)
            icrc = d_icrc.cpu().numpy().view(np.uint32)
            fr = d_frames.cpu().numpy().reshape(npkts, slot)
            assert not d_st.cpu().numpy().any()
            for p, f in enumerate(want):
                assert lens[p] == len(f), p
                assert fr[p, : len(f)].tobytes() == f, p
                assert icrc[p] == O.icrc_of_frame(f), p
    finally:
        engine.set_lanes(0)

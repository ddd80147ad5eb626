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


def _check_against_oracle(eng, mr: bytes, wrs, pmtu):
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
        tail = (-len(f)) % 16  # slot bytes up to the next 16-byte boundary are zero
        assert not frames[p, len(f): len(f) + tail].any()


@pytest.mark.parametrize("pmtu", (256, 1024, 4096))
@pytest.mark.parametrize("lanes", (0, 2, 4, 8, 16))
def test_every_op_and_boundary_length(engine, pmtu, lanes):
    mr = np.random.default_rng(pmtu + lanes).integers(0, 256, 5 * pmtu + 7, dtype=np.uint8).tobytes()
    wrs = all_ops_cases(pmtu, len(mr), seed=pmtu * 7 + lanes)
    engine.set_lanes(lanes)
    try:
        _check_against_oracle(engine, mr, wrs, pmtu)
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
    rec2[2]["op"] = 9
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

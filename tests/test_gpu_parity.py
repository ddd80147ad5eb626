"""GPU parity: the HIP ICRC engine (through the C ABI) against the CPU oracle.

Bar: bit-exact uint32 ICRC words for every frame.  The oracle restates
BTH.compute_icrc (datenlord/roce-sim src/roce.py:192-223); see oracle/.
"""
import numpy as np
import pytest

from conftest import oracle_batch

pytestmark = pytest.mark.gpu

import icrc_oracle as o  # noqa: E402  (checker only)
from roce_icrc import synth  # noqa: E402
from roce_icrc.engine import (  # noqa: E402
    PKT_BAD_LEN, PKT_FATAL, PKT_ICRC_MISMATCH, PKT_LEN_MISMATCH, PKT_NOT_IPV4, PKT_NOT_UDP)

LANES = [1, 2, 4, 8, 16, 32, 64]


def _opcode_frames():
    """One frame per (opcode shape, payload length) the simulator emits
    (src/roce_sq.py:1243-1466, src/roce_rq.py:388-525, 767-854)."""
    rng = np.random.default_rng(7)
    frames = []
    ext_for = {
        0x00: b"", 0x01: b"", 0x02: b"", 0x04: b"",
        0x03: o.immdt_bytes(0x1234), 0x05: o.immdt_bytes(0xBEEF),
        0x06: o.reth_bytes(0x1000, 0x55, 4096), 0x07: b"", 0x08: b"",
        0x09: o.immdt_bytes(7), 0x0A: o.reth_bytes(0x2000, 0x66, 100),
        0x0B: o.reth_immdt_bytes(0x3000, 0x77, 10, 0x99),
        0x0C: o.reth_bytes(0x4000, 0x88, 8192),
        0x0D: o.aeth_bytes(0, 31, 5), 0x0E: b"", 0x0F: o.aeth_bytes(0, 31, 6),
        0x10: o.aeth_bytes(0, 31, 7), 0x11: o.aeth_bytes(3, 2, 9),
        0x12: o.aeth_bytes(0, 31, 3) + o.atomic_ack_eth_bytes(0x1122334455667788),
        0x13: o.atomic_eth_bytes(0x5000, 0x1, 5, 6), 0x14: o.atomic_eth_bytes(0x6000, 0x2, 0, 9),
        0x16: o.ieth_bytes(0xAB), 0x17: o.ieth_bytes(0xCD),
        0x81: o.cnp_padding_bytes(),
    }
    no_payload = {0x0C, 0x11, 0x12, 0x13, 0x14, 0x81}
    for op, ext in ext_for.items():
        plens = [None] if op in no_payload else [0, 1, 2, 3, 4, 5, 255, 256, 1023, 4096]
        for pl in plens:
            payload = None if pl is None else rng.integers(0, 256, pl, dtype=np.uint8).tobytes()
            frames.append(o.build_frame("192.168.0.1", "192.168.0.2", 0x33,
                                        dict(opcode=op, psn=int(rng.integers(1 << 24)),
                                             dqpn=0x11, ackreq=int(op & 1)),
                                        ext=ext, payload=payload))
    return frames


def _pack(frames, align=4):
    offs, pos = [], 0
    for f in frames:
        offs.append(pos)
        pos += (len(f) + align - 1) // align * align
    buf = np.zeros(pos, np.uint8)
    for off, f in zip(offs, frames):
        buf[off:off + len(f)] = np.frombuffer(f, np.uint8)
    return buf, np.array(offs, np.uint64), np.array([len(f) for f in frames], np.uint32)


def test_cfg1_sim_send_success(engine):
    """Config 1: the sim_send_success SEND_ONLY; known value from SURVEY App. B."""
    f = o.sim_send_success_frame()
    icrc, st = engine.compute_one(f)
    assert st == 0
    assert icrc == 0x1BE21D75 == o.icrc_of_frame(f)
    assert f[-4:] == bytes.fromhex("751de21b")


@pytest.mark.parametrize("lanes", LANES)
def test_every_opcode_shape(engine, lanes):
    frames = _opcode_frames()
    buf, offs, lens = _pack(frames)
    engine.set_lanes(lanes)
    try:
        got, st = engine.compute_batch(buf, offs, lens)
    finally:
        engine.set_lanes(0)
    want = np.array([o.icrc_of_frame(f) for f in frames], np.uint32)
    assert (st & 0x07 == 0).all()
    np.testing.assert_array_equal(got, want)
    ok, got2, _ = engine.verify_batch(buf, offs, lens)
    assert ok.all()
    np.testing.assert_array_equal(got2, want)


@pytest.mark.parametrize("lanes", LANES)
def test_uniform_4k_strided(engine, lanes):
    n = 3000
    buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
    engine.set_lanes(lanes)
    try:
        got, st = engine.compute_strided(buf, stride, flen, n)
    finally:
        engine.set_lanes(0)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    assert (st == 0).all()
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("n", [1, 7, 257, 1283, 9001, 40003])
def test_strided_batch_sizes_output_runs(engine, n):
    """The strided kernel writes a workgroup's ICRC words as one run of
    16-byte buffer stores plus a 4-byte remainder (round 2); tail sets
    claimed from other workgroups write their own words.  Batch sizes that
    leave every remainder length, at 1, 8 and 64 lanes, bit-exact and with
    nothing written past the batch."""
    buf, stride, flen = synth.uniform_frames(n, 512, seed=synth.SEED_CFG2 + n)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    for lanes in (1, 8, 64):
        engine.set_lanes(lanes)
        try:
            got, st = engine.compute_strided(buf, stride, flen, n)
        finally:
            engine.set_lanes(0)
        assert (st == 0).all()
        np.testing.assert_array_equal(got, want, err_msg=f"lanes {lanes}")
    torch = pytest.importorskip("torch")
    d = torch.from_numpy(buf).cuda()
    out = torch.full((n + 64,), -1, dtype=torch.int32, device="cuda")  # sentinel tail
    engine.compute_strided_dev(d, stride, flen, n, out)
    torch.cuda.synchronize()
    h = out.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(h[:n], want)
    assert (h[n:] == 0xFFFFFFFF).all()


@pytest.mark.parametrize("lanes", LANES)
def test_mixed_mtu_compute_and_verify(engine, lanes):
    n = 5000
    buf, offs, lens = synth.mixed_mtu_frames(n, seed=synth.SEED_CFG3)
    want, _ = oracle_batch(buf, offs, lens)
    # fill trailers (little-endian ICRC) so verify has correct frames
    for i in range(n):
        e = int(offs[i] + lens[i])
        buf[e - 4:e] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    rng = np.random.default_rng(3)
    bad = rng.choice(n, 40, replace=False)
    flip, masked = bad[:20], bad[20:]
    for i in flip:  # payload bit flip: must fail
        p = int(offs[i]) + 40 + int(rng.integers(0, lens[i] - 44))
        buf[p] ^= np.uint8(1 << int(rng.integers(0, 8)))
    for i in masked:  # random values in masked fields: must still pass
        b = int(offs[i])
        for k in (1, 8, 10, 11, 26, 27, 32):
            buf[b + k] = rng.integers(0, 256)
    engine.set_lanes(lanes)
    try:
        got, st = engine.compute_batch(buf, offs, lens)
        ok, got2, st2 = engine.verify_batch(buf, offs, lens)
    finally:
        engine.set_lanes(0)
    want2, ok_want = oracle_batch(buf, offs, lens)
    np.testing.assert_array_equal(got, want2)
    np.testing.assert_array_equal(got2, want2)
    np.testing.assert_array_equal(ok, ok_want.astype(bool))
    assert not ok[flip].any()
    assert ok[masked].all()
    assert (st2[flip] & PKT_ICRC_MISMATCH).all()
    assert ok.sum() == n - len(flip)


def test_small_packets_cfg5_shape(engine):
    n = 40000
    buf, stride, flen = synth.uniform_frames(n, 64, seed=synth.SEED_CFG5)
    got, st = engine.compute_strided(buf, stride, flen, n)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    np.testing.assert_array_equal(got, want)


def test_edge_cases_and_status(engine):
    good = o.build_frame("1.2.3.4", "5.6.7.8", 9, dict(opcode=0x11, psn=5), ext=o.aeth_bytes())
    bare = o.build_frame("1.2.3.4", "5.6.7.8", 9, dict(opcode=0x01, psn=5))  # 44 B minimum
    assert len(bare) == 44
    not_ip = b"\x60" + good[1:]          # IPv6 version nibble
    not_udp = good[:9] + b"\x06" + good[10:]  # TCP protocol
    short = good[:40]                    # shorter than IP+UDP+BTH+ICRC
    odd = good + b"\0\0"                 # length not a multiple of 4 (CRC'd, as zlib would)
    mism = good[:2] + b"\x00\x10" + good[4:]  # IP total length != frame length
    # IPv4 with options (IHL 6): masks move with the UDP/BTH offsets
    opt = bytearray(good[:20]) + b"\x01\x01\x01\x01" + good[20:]
    opt[0] = 0x46
    opt[2:4] = len(opt).to_bytes(2, "big")
    opt = bytes(opt)
    frames = [good, bare, not_ip, not_udp, short, odd, mism, opt]
    buf, offs, lens = _pack(frames)
    got, st = engine.compute_batch(buf, offs, lens)
    assert got[0] == o.icrc_of_frame(good) and st[0] == 0
    assert got[1] == o.icrc_of_frame(bare) and st[1] == 0
    assert got[2] == 0 and st[2] & PKT_NOT_IPV4
    assert got[3] == 0 and st[3] & PKT_NOT_UDP
    assert got[4] == 0 and st[4] & PKT_BAD_LEN
    assert got[5] == o.icrc_of_frame(odd) != 0 and st[5] == PKT_LEN_MISMATCH
    assert got[6] == o.icrc_of_frame(mism) and st[6] == PKT_LEN_MISMATCH
    assert got[7] == o.icrc_of_frame(opt) and st[7] == 0
    # empty batch and single frame at the very end of the buffer
    e0, s0 = engine.compute_batch(np.zeros(0, np.uint8), np.zeros(0, np.uint64),
                                  np.zeros(0, np.uint32))
    assert e0.size == 0
    icrc, st1 = engine.compute_one(bare)
    assert icrc == o.icrc_of_frame(bare)


def test_unaligned_offsets(engine):
    """Frames at every dword alignment modulo 16 and 128 bytes."""
    rng = np.random.default_rng(11)
    frames = [o.build_frame("10.0.0.1", "10.0.0.2", 3, dict(opcode=0x07, psn=i),
                            payload=rng.integers(0, 256, int(rng.integers(0, 600)) * 4,
                                                 dtype=np.uint8).tobytes())
              for i in range(257)]
    buf, offs, lens = _pack(frames, align=4)
    assert len({int(x) % 16 for x in offs}) == 4
    for lanes in (1, 16, 64):
        engine.set_lanes(lanes)
        got, _ = engine.compute_batch(buf, offs, lens)
        np.testing.assert_array_equal(got, [o.icrc_of_frame(f) for f in frames])
    engine.set_lanes(0)


def test_maximum_length_frames(engine):
    """IPv4's largest frame that is a multiple of 4 (65532 B: 16383 dwords, 2047
    lane-group iterations at G = 8) between small ones, ragged and strided,
    compute and verify; 65536 B exceeds the IPv4 total length and is flagged."""
    rng = np.random.default_rng(65532)
    big = o.build_frame("10.0.0.1", "10.0.0.2", 5, dict(opcode=0x07, psn=1),
                        payload=rng.integers(0, 256, 65532 - 44, dtype=np.uint8).tobytes())
    assert len(big) == 65532
    small = o.build_frame("10.0.0.1", "10.0.0.2", 5, dict(opcode=0x07, psn=2), payload=b"\1" * 64)
    over = bytearray(big + b"\0\0\0\0")  # 65536 B: no valid IPv4 total length
    frames = [small, big, small, big, bytes(over), small]
    buf, offs, lens = _pack(frames)
    want = [o.icrc_of_frame(f) for f in frames[:4]] + [0, o.icrc_of_frame(small)]
    for lanes in (0, 8, 64):
        engine.set_lanes(lanes)
        got, st = engine.compute_batch(buf, offs, lens)
        np.testing.assert_array_equal(got, want)
        assert st[4] & PKT_BAD_LEN and (np.delete(st, 4) == 0).all()
        for i in range(4):
            e = int(offs[i] + lens[i])
            buf[e - 4:e] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
        ok, _, _ = engine.verify_batch(buf, offs, lens)
        assert ok[:4].all() and not ok[4]
        sbuf = np.frombuffer(big * 3, np.uint8).copy()
        got, st = engine.compute_strided(sbuf, len(big), len(big), 3)
        assert (got == want[1]).all() and (st == 0).all()
    engine.set_lanes(0)


@pytest.mark.parametrize("lanes", [0, 1, 8, 64])
def test_misaligned_frames(engine, lanes):
    """Frames whose start is not 4-byte aligned get their real ICRC, like the
    reference's zlib.crc32 wherever the bytes sit (byte-load slow path), in
    compute and verify, on the staged small-call path and on a large batch;
    the aligned neighbours are unaffected and the multi-GPU entry point (which
    realigns while gathering) agrees."""
    from roce_icrc import compute_batch_multi
    rng = np.random.default_rng(3 + lanes)
    frames = [o.build_frame("1.2.3.4", "5.6.7.8", 9, dict(opcode=0x04, psn=i),
                            payload=rng.integers(0, 256, int(rng.integers(0, 1100)),
                                                 dtype=np.uint8).tobytes())
              for i in range(40)]
    frames[7] = o.build_frame("1.2.3.4", "5.6.7.8", 9, dict(opcode=0x04, psn=7))  # 44 B minimum
    want = np.array([o.icrc_of_frame(f) for f in frames], np.uint32)
    engine.set_lanes(lanes)
    try:
        for reps in (1, 80):  # 80 x 40 frames: past the pinned staging block
            fs = frames * reps
            buf = np.zeros(sum(len(f) + 8 for f in fs) + 8, np.uint8)
            offs, pos = [], 0
            for i, f in enumerate(fs):
                pos += i % 4  # every byte misalignment, in turn
                buf[pos:pos + len(f)] = np.frombuffer(f, np.uint8)
                offs.append(pos)
                pos += len(f)
            offs = np.array(offs, np.uint64)
            lens = np.array([len(f) for f in fs], np.uint32)
            assert len({int(x) % 4 for x in offs}) == 4
            got, st = engine.compute_batch(buf, offs, lens)
            np.testing.assert_array_equal(got, np.tile(want, reps))
            assert (st == 0).all()
            got_m, st_m = compute_batch_multi([engine, engine], buf, offs, lens)
            np.testing.assert_array_equal(got_m, got)
            np.testing.assert_array_equal(st_m, st)
            for i, f in enumerate(fs):
                e = int(offs[i]) + len(f)
                buf[e - 4:e] = np.frombuffer(int(want[i % 40]).to_bytes(4, "little"), np.uint8)
            bad = [5, 6, 22, 23]  # one per misalignment: a payload bit flip must fail
            for i in bad:
                buf[int(offs[i]) + 40] ^= 0x10
            ok, got2, st2 = engine.verify_batch(buf, offs, lens)
            expect = np.ones(len(fs), bool)
            expect[bad] = False
            np.testing.assert_array_equal(ok, expect)
            assert (st2[bad] & PKT_ICRC_MISMATCH).all()
    finally:
        engine.set_lanes(0)


def test_misaligned_frames_device_resident(engine):
    """The device-resident ragged entry points and a strided batch whose
    stride is not a multiple of 4 (every other frame unaligned)."""
    import torch
    rng = np.random.default_rng(17)
    frames = [o.build_frame("10.0.0.1", "10.0.0.2", 3, dict(opcode=0x07, psn=i),
                            payload=rng.integers(0, 256, 4 * int(rng.integers(0, 300)),
                                                 dtype=np.uint8).tobytes())
              for i in range(3000)]
    want = np.array([o.icrc_of_frame(f) for f in frames], np.uint32)
    buf = np.zeros(sum(len(f) + 3 for f in frames), np.uint8)
    offs, pos = [], 0
    for i, f in enumerate(frames):
        pos += i % 4
        buf[pos:pos + len(f)] = np.frombuffer(f, np.uint8)
        offs.append(pos)
        pos += len(f)
    lens = np.array([len(f) for f in frames], np.uint32)
    d_buf = torch.from_numpy(buf).cuda()
    d_offs = torch.from_numpy(np.array(offs, np.int64)).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(len(frames), dtype=torch.int32, device="cuda")
    st = torch.zeros(len(frames), dtype=torch.uint8, device="cuda")
    engine.compute_batch_dev(d_buf, d_offs, d_lens, len(frames), out, st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    assert (st.cpu().numpy() == 0).all()
    # strided: 2 + 4140-B stride, so frame i starts at 2 i (mod 4)
    sb, stride, flen = synth.uniform_frames(64, 4096, seed=5)
    f2 = [sb[i * stride:i * stride + flen].tobytes() for i in range(64)]
    s2 = flen + 2
    buf2 = np.zeros(64 * s2, np.uint8)
    for i, f in enumerate(f2):
        buf2[i * s2:i * s2 + flen] = np.frombuffer(f, np.uint8)
    got, st2 = engine.compute_strided(buf2, s2, flen, 64)
    np.testing.assert_array_equal(got, [o.icrc_of_frame(f) for f in f2])
    assert (st2 == 0).all()


def test_mask_invariance_and_sensitivity(engine):
    base = o.build_frame("10.9.8.7", "10.6.5.4", 17, dict(opcode=0x0A, psn=99, dqpn=0x42),
                         ext=o.reth_bytes(1, 2, 3), payload=bytes(range(200)))
    rng = np.random.default_rng(5)
    variants = [base]
    for _ in range(64):  # masked fields randomised: same ICRC
        b = bytearray(base)
        for k in (1, 8, 10, 11, 26, 27, 32):
            b[k] = int(rng.integers(0, 256))
        variants.append(bytes(b))
    sens = []
    for k in (4, 5, 6, 7, 30, 31, 36, 40, 100, len(base) - 5):  # id, flags, pkey, ackreq, data
        b = bytearray(base)
        b[k] ^= 0x01
        sens.append(bytes(b))
    buf, offs, lens = _pack(variants + sens)
    got, _ = engine.compute_batch(buf, offs, lens)
    ref = o.icrc_of_frame(base)
    assert (got[:len(variants)] == ref).all()
    assert (got[len(variants):] != ref).all()
    np.testing.assert_array_equal(got[len(variants):], [o.icrc_of_frame(f) for f in sens])


def test_device_resident_torch(engine):
    torch = pytest.importorskip("torch")
    n = 2048
    buf, stride, flen = synth.uniform_frames(n, 4096, seed=1)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    engine.compute_strided_dev(d, stride, flen, n, out, st, stream=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    # write the trailers on the device, then verify there
    rows = d.view(n, stride)
    rows[:, flen - 4:flen] = out.view(torch.uint8).view(n, 4)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_strided_dev(d, stride, flen, n, ok, stream=s.cuda_stream)
    s.synchronize()
    assert bool(ok.all())
    rows[7, 100] ^= 1
    engine.verify_strided_dev(d, stride, flen, n, ok, stream=s.cuda_stream)
    s.synchronize()
    okc = ok.cpu().numpy()
    assert okc[7] == 0 and okc.sum() == n - 1


def test_strided_tail_claims_concurrent_streams(engine):
    """The strided kernel's workgroups claim the tails of their ranges (and of
    other workgroups' ranges) through per-context counters: launches of ONE
    context in flight on several streams at once, and many back-to-back
    launches (counter slots reused every 64 epochs), stay bit-exact; so do
    batch sizes whose ranges are shorter than a tail (few sets per block)."""
    torch = pytest.importorskip("torch")
    sizes = [1 << 16, 3 * 257 + 5, 8 * 256 * 4 + 1, 77]
    data = []
    for i, n in enumerate(sizes):
        buf, stride, flen = synth.uniform_frames(n, 4096, seed=40 + i)
        want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
        data.append((torch.from_numpy(buf).cuda(), stride, flen, n, want))
    streams = [torch.cuda.Stream() for _ in sizes]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _, _, _, n, _ in data]
    torch.cuda.synchronize()
    for rep in range(40):  # 160 launches: every claim slot is reused
        for (d, stride, flen, n, _), out, st in zip(data, outs, streams):
            engine.compute_strided_dev(d, stride, flen, n, out, stream=st.cuda_stream)
    torch.cuda.synchronize()
    for (_, _, _, _, want), out in zip(data, outs):
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)


def test_claim_counters_never_shared_by_concurrent_launches(engine):
    """One long strided launch on stream A while more than 64 short launches of
    the SAME context go to three other streams (3 does not divide the 64 claim
    slots): a launch must never find its tail-claim counters overwritten by a
    launch in flight on another stream (which would leave its tail sets
    unprocessed and their words stale).  Every output against the oracle."""
    torch = pytest.importorskip("torch")
    n_long = 1 << 20
    buf, stride, flen = synth.uniform_frames(n_long, 4096, seed=77)
    want_long, _ = oracle_batch(buf, stride=stride, length=flen, n=n_long)
    d_long = torch.from_numpy(buf).cuda()
    del buf
    shorts = []
    for i, n in enumerate([8 * 256 * 4 + 1, 8 * 256 * 4 + 77, 3 * 8 * 256 + 5]):
        b, s_, f_ = synth.uniform_frames(n, 4096, seed=80 + i)
        w, _ = oracle_batch(b, stride=s_, length=f_, n=n)
        shorts.append((torch.from_numpy(b).cuda(), s_, f_, n, w))
    out_long = torch.full((n_long,), -1, dtype=torch.int32, device="cuda")
    outs = [torch.full((n,), -1, dtype=torch.int32, device="cuda") for *_, n, _ in shorts]
    sa = torch.cuda.Stream()
    ss = [torch.cuda.Stream() for _ in shorts]
    torch.cuda.synchronize()
    for rep in range(3):
        out_long.fill_(-1)
        torch.cuda.synchronize()
        engine.compute_strided_dev(d_long, stride, flen, n_long, out_long, stream=sa.cuda_stream)
        for _ in range(30):  # 90 short launches behind the long one
            for (d, s_, f_, n, _), out, st in zip(shorts, outs, ss):
                engine.compute_strided_dev(d, s_, f_, n, out, stream=st.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out_long.cpu().numpy().view(np.uint32), want_long)
        for (*_, w), out in zip(shorts, outs):
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), w)


def test_multi_context_round_robin(engine):
    from roce_icrc import IcrcEngine, compute_batch_multi
    n = 3001
    buf, offs, lens = synth.mixed_mtu_frames(n, seed=9)
    e2 = IcrcEngine(0)
    try:
        got, _ = compute_batch_multi([engine, e2, e2], buf, offs, lens)
    finally:
        e2.close()
    want, _ = oracle_batch(buf, offs, lens)
    np.testing.assert_array_equal(got, want)


def test_multi_chunked_compute_and_verify(engine):
    """The multi split streams each shard in chunks (8 MiB of frames or 65536
    packets) through two pinned blocks: shards of many chunks, a chunk boundary
    inside a run of ACK-sized frames, odd lengths, and one 9 MiB non-frame
    (status BAD_LEN, ICRC 0) that forces the blocks to grow.  compute and
    verify through the C ABI against the oracle; verify flags exactly the
    corrupted frames (src/roce_v2.py:327-372 is the receive batch it serves)."""
    from roce_icrc import IcrcEngine, compute_batch_multi, verify_batch_multi
    big_buf, big_offs, big_lens = synth.mixed_mtu_frames(30000, seed=21)
    tiny_buf, tiny_offs, tiny_lens = synth.mixed_mtu_frames(300000, seed=22, mtus=(0,))
    huge = np.random.default_rng(3).integers(0, 256, 9 << 20, dtype=np.uint8)
    parts = [(big_buf, big_offs, big_lens), (tiny_buf, tiny_offs, tiny_lens),
             (huge, np.zeros(1, np.uint64), np.array([huge.size], np.uint32))]
    buf = np.concatenate([p[0] for p in parts])
    base = np.cumsum([0] + [p[0].size for p in parts[:-1]]).astype(np.uint64)
    offs = np.concatenate([p[1] + b for p, b in zip(parts, base)])
    lens = np.concatenate([p[2] for p in parts]).astype(np.uint32)
    lens[7] -= 2  # odd length (CRC'd as zlib would; IP length mismatch status)
    rng = np.random.default_rng(5)
    perm = rng.permutation(offs.size)  # interleave the families across shards
    offs, lens = offs[perm], lens[perm]
    want, _ = oracle_batch(buf, offs, lens)
    good = lens <= 65535  # (the 9 MiB one: the reference's "warning + ICRC 0" path)
    assert (~good).sum() == 1 and want[~good][0] == 0
    e2 = IcrcEngine(0)
    try:
        got, st = compute_batch_multi([engine, e2, e2], buf, offs, lens)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal((st & PKT_FATAL) != 0, ~good)
        assert st[np.flatnonzero(perm == 7)[0]] == PKT_LEN_MISMATCH
        # stamp the answers, corrupt 97 frames, verify on the same split
        for i in range(offs.size):
            e = int(offs[i]) + int(lens[i])
            if lens[i] <= 65535 and lens[i] >= 4:
                buf[e - 4:e] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
        bad = rng.choice(np.flatnonzero(good), 97, replace=False)
        for i in bad:
            buf[int(offs[i]) + int(lens[i]) - 1] ^= 0x40  # the ICRC trailer's top byte
        ok, icrc, st2 = verify_batch_multi([e2, engine], buf, offs, lens)
        want_ok = good.copy()
        want_ok[bad] = False
        np.testing.assert_array_equal(ok, want_ok)
        np.testing.assert_array_equal(icrc, want)
        assert ((st2 & PKT_ICRC_MISMATCH) != 0).sum() == 97
    finally:
        e2.close()


def test_full_size_cfg2_bit_exact(engine):
    """BASELINE config 2 at full size (2^20 x 4 KiB frames): every ICRC word
    against the multi-threaded C oracle."""
    torch = pytest.importorskip("torch")
    n = 1 << 20
    buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.compute_strided_dev(d, stride, flen, n, out, stream=s.cuda_stream)
    s.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    del d
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    np.testing.assert_array_equal(got, want)


def test_full_size_cfg3_ragged_bit_exact(engine):
    """BASELINE config 3 at full size (2^20 mixed-MTU frames, several sort
    windows per workgroup): every ICRC word and verdict against the C oracle,
    packed in memory order and with the descriptors shuffled (frames in
    arbitrary order, so the block-local sort sees scattered offsets)."""
    torch = pytest.importorskip("torch")
    n = 1 << 20
    buf, offs, lens = synth.mixed_mtu_frames(n)
    want, _ = oracle_batch(buf, offsets=offs, lens=lens)
    d = torch.from_numpy(buf).cuda()
    s = torch.cuda.current_stream()
    perm = np.random.default_rng(3).permutation(n)
    for o, l in ((offs, lens), (offs[perm], lens[perm])):
        do = torch.from_numpy(np.ascontiguousarray(o).view(np.int64)).cuda()
        dl = torch.from_numpy(np.ascontiguousarray(l).view(np.int32)).cuda()
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        engine.compute_batch_dev(d, do, dl, n, out, stream=s.cuda_stream)
        s.synchronize()
        exp = want if o is offs else want[perm]
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
    # trailers filled with the words: every verdict passes, then one byte of
    # every 997th frame flipped (past its 40-byte header): those fail
    trail = offs.astype(np.int64) + lens.astype(np.int64) - 4
    idx = (trail[:, None] + np.arange(4)[None, :]).reshape(-1)
    buf[idx] = want.view(np.uint8)
    bad = np.arange(0, n, 997)
    buf[offs[bad].astype(np.int64) + 44] ^= 0x40
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch_dev(d, do, dl, n, ok, stream=s.cuda_stream)
    s.synchronize()
    okh = ok.cpu().numpy().astype(bool)
    expect = np.ones(n, bool)
    expect[bad] = False
    np.testing.assert_array_equal(okh, expect)


def test_full_size_cfg5_small_bit_exact(engine):
    """BASELINE config 5 at full size (2^24 x 108-B frames, the lane-per-packet
    kernel including its direct last batch): every word against the C oracle."""
    torch = pytest.importorskip("torch")
    n = 1 << 24
    buf, stride, flen = synth.uniform_frames(n, 64, seed=synth.SEED_CFG5)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.compute_strided_dev(d, stride, flen, n, out, stream=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("n", [256 * 486 * 64 - 1000, 256 * 458 * 64 + 77])
def test_small_kernel_many_ring_windows(engine, n):
    """~7.5 M 108-B frames put 40.5 / 38.2 rounds of 12 batches on each
    workgroup of the small kernel: several full output-ring windows, then a
    last window ending with a round that only some waves of the workgroup
    have.  (Round 3 measured a register extension of the window here,
    scratch/attic/small_register_rounds.diff; this case caught its first
    version, whose idle waves skipped a shift.)"""
    torch = pytest.importorskip("torch")
    buf, stride, flen = synth.uniform_frames(n, 64, seed=0x5A11)
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.compute_strided_dev(d, stride, flen, n, out, stream=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("payload,stride", [(4, 48), (76, 128)])
def test_small_kernel_ring_regions(engine, payload, stride):
    """The small-frame kernel's output ring starts in the free halves of its
    table rows and continues after the staging slots (round 2).  Batches
    large enough that every workgroup's flushes run through both regions, at
    the smallest stride (12 waves) and the largest (10 waves after rounding
    to even, the largest per-wave slot), with a gap after each frame at 128:
    every word against the C oracle, nothing written past the batch."""
    torch = pytest.importorskip("torch")
    n = 6_000_011  # > 256 workgroups x 2 full rings of 128-B frames
    flen = 44 + payload
    frames, s0, _ = synth.uniform_frames(n, payload, seed=synth.SEED_CFG5 + stride)
    buf = np.zeros((n - 1) * stride + flen, np.uint8)
    rows = np.lib.stride_tricks.as_strided(buf, (n, flen), (stride, 1))
    rows[:] = frames.reshape(n, s0)[:, :flen]
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
    d = torch.from_numpy(buf).cuda()
    out = torch.full((n + 256,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.compute_strided_dev(d, stride, flen, n, out, stream=s.cuda_stream)
    s.synchronize()
    h = out.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(h[:n], want)
    assert (h[n:] == 0xFFFFFFFF).all()


def test_ragged_many_windows_random_sizes(engine):
    """The ragged kernels over 3 x 2^20 frames of random length (44 .. 1020 B,
    so every workgroup sorts several windows -- two of 6144 in the
    mixed-width kernel, whose windows hold up to 8192 -- and claims sets from
    both ends of each), laid out in memory order with malformed frames
    scattered in: lengths not a multiple of 4 (CRC'd through the byte-load
    path, as zlib.crc32 would), TCP instead of UDP, an IP total
    length that disagrees with the frame, IPv4 options.  Lane settings 4, 8
    (the mixed-width kernel: G = 4 and G = 8 sets) and 16; compute and verify
    against the C oracle."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(2024)
    n = 3 << 20
    lens = (rng.integers(11, 256, n) * 4).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], out=offs[1:])
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1]), dtype=np.uint8)
    o64 = offs.astype(np.int64)
    buf[o64] = 0x45
    tot = lens.copy()
    mism = rng.choice(n, 500, replace=False)
    tot[mism] += 4
    buf[o64 + 2] = (tot >> 8).astype(np.uint8)
    buf[o64 + 3] = (tot & 0xFF).astype(np.uint8)
    buf[o64 + 9] = 17
    tcp = rng.choice(n, 500, replace=False)
    buf[o64[tcp] + 9] = 6
    opt = rng.choice(n, 500, replace=False)
    buf[o64[opt]] = 0x46
    odd = rng.choice(n, 500, replace=False)
    lens_k = lens.copy()
    lens_k[odd] -= (2 + 4 * (odd % 3)).astype(np.uint32)  # 2 / 6 / 10 bytes early: not a multiple of 4
    want, _ = oracle_batch(buf, offsets=offs, lens=lens)
    # trailers = the oracle's words (frames it rejects keep 0 there, and so
    # fail verification like on the GPU); then one payload bit of every 1013th
    trail = o64 + lens.astype(np.int64) - 4
    buf[(trail[:, None] + np.arange(4)[None, :]).reshape(-1)] = want.view(np.uint8)
    flip = np.arange(5, n, 1013)
    buf[o64[flip] + 40] ^= 0x08
    # the oracle over the lengths the GPU is given (odd ones included: any
    # length is CRC'd, as zlib.crc32 does; their trailers do not match)
    want, ok_want = oracle_batch(buf, offsets=offs, lens=lens_k)
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens_k.view(np.int32)).cuda()
    s = torch.cuda.current_stream()
    for lanes in (4, 8, 16):
        engine.set_lanes(lanes)
        try:
            out = torch.zeros(n, dtype=torch.int32, device="cuda")
            ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
            engine.compute_batch_dev(d, do, dl, n, out, stream=s.cuda_stream)
            engine.verify_batch_dev(d, do, dl, n, ok, stream=s.cuda_stream)
            s.synchronize()
        finally:
            engine.set_lanes(0)
        got = out.cpu().numpy().view(np.uint32)
        okh = ok.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(got, want, err_msg=f"lanes {lanes}")
        assert not okh[odd].any()  # (their trailers do not match)
        np.testing.assert_array_equal(okh, ok_want.astype(bool), err_msg=f"lanes {lanes}")
        assert not okh[flip].any() and okh.sum() > n - 5000


@pytest.mark.parametrize("mtus,n", [
    ((548, 552, 556, 560, 564, 568), 200_003),   # frames 592 .. 612 B: the width boundary (600 B)
    ((4, 4096), 100_001),                          # tiny and 4-KiB frames alternate in memory
    ((8,) * 15 + (4096,), 300_007),               # one long frame per 16 short ones
    ((256, 512, 1024, 2048, 4096), 2_200_009),    # cfg3 mix, two windows per workgroup
])
def test_mixed_width_claims(engine, mtus, n):
    """The mixed-width ragged kernel (the lanes-8 / device-resident default):
    claims of 16 short sorted frames run as one G = 4 set, the rest as G = 8
    sets of 8, from both ends of every window.  Compositions that put the
    600-B width boundary inside claims, alternate tiny and 4-KiB frames, or
    hold one long frame per 16 short ones, with batch sizes that leave
    partial claims where the two ends meet; compute and verify against the C
    oracle (every 101st frame's payload corrupted for verify)."""
    torch = pytest.importorskip("torch")
    buf, offs, lens = synth.mixed_mtu_frames(n, mtus=mtus, seed=n)
    want, _ = oracle_batch(buf, offsets=offs, lens=lens)
    s = torch.cuda.current_stream()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    engine.set_lanes(8)
    try:
        d = torch.from_numpy(buf).cuda()
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        engine.compute_batch_dev(d, do, dl, n, out, stream=s.cuda_stream)
        s.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
        trail = offs.astype(np.int64) + lens.astype(np.int64) - 4
        buf[(trail[:, None] + np.arange(4)[None, :]).reshape(-1)] = want.view(np.uint8)
        bad = np.arange(3, n, 101)
        buf[offs[bad].astype(np.int64) + 41] ^= 0x10
        d = torch.from_numpy(buf).cuda()
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        engine.verify_batch_dev(d, do, dl, n, ok, stream=s.cuda_stream)
        s.synchronize()
    finally:
        engine.set_lanes(0)
    expect = np.ones(n, bool)
    expect[bad] = False
    np.testing.assert_array_equal(ok.cpu().numpy().astype(bool), expect)


@pytest.mark.parametrize("n", [37, 20_011, 600_001])
def test_host_ragged_tiny_frames(engine, n):
    """Host-buffer ragged batches whose mean frame is <= 128 B (ACK-sized
    48-B frames with a few 4-KiB ones mixed in) run one lane per packet
    (ragged_log2g): compute and verify against the C oracle, through the
    pinned staging block (small calls) and the device scratch (large)."""
    rng = np.random.default_rng(n)
    mtus = (4,) * 63 + (4096,)
    buf, offs, lens = synth.mixed_mtu_frames(n, mtus=mtus, seed=n)
    assert lens.mean() <= 128 or n < 64
    want, _ = oracle_batch(buf, offsets=offs, lens=lens)
    got, st = engine.compute_batch(buf, offs, lens)
    np.testing.assert_array_equal(got, want)
    assert (st == 0).all()
    trail = offs.astype(np.int64) + lens.astype(np.int64) - 4
    buf[(trail[:, None] + np.arange(4)[None, :]).reshape(-1)] = want.view(np.uint8)
    bad = rng.choice(n, max(1, n // 97), replace=False)
    buf[offs[bad].astype(np.int64) + 40] ^= 0x01
    ok, got2, _ = engine.verify_batch(buf, offs, lens)
    expect = np.ones(n, bool)
    expect[bad] = False
    np.testing.assert_array_equal(ok, expect)


def test_offsets_above_16_gib(engine):
    """Frames placed beyond 2^34 bytes into one 17-GiB device buffer.  The
    ragged kernel keeps sorted offsets as u32 dwords (< 16 GiB) and takes a
    larger offset from the descriptor array in HBM instead; this interleaves
    both kinds in every sort window, for compute and verify, at lanes 4/8/16,
    against the C oracle (the HBM layout is sized for 288 GB per GPU)."""
    torch = pytest.importorskip("torch")
    n = 20000
    lo_buf, lo_offs, lens_a = synth.mixed_mtu_frames(n, seed=41)
    hi_buf, hi_offs, lens_b = synth.mixed_mtu_frames(n, seed=42)
    want_a, _ = oracle_batch(lo_buf, offsets=lo_offs, lens=lens_a)
    want_b, _ = oracle_batch(hi_buf, offsets=hi_offs, lens=lens_b)
    hi0 = (1 << 34) + 4096 + 12  # dword- but not 16-byte-aligned base
    d = torch.empty(hi0 + hi_buf.size, dtype=torch.uint8, device="cuda")
    d[:lo_buf.size].copy_(torch.from_numpy(lo_buf))
    d[hi0:hi0 + hi_buf.size].copy_(torch.from_numpy(hi_buf))
    offs = np.empty(2 * n, np.uint64)
    offs[0::2] = lo_offs
    offs[1::2] = hi_offs + np.uint64(hi0)
    lens = np.empty(2 * n, np.uint32)
    lens[0::2], lens[1::2] = lens_a, lens_b
    want = np.empty(2 * n, np.uint32)
    want[0::2], want[1::2] = want_a, want_b
    # trailers = the words, then one payload bit of every 101st frame flipped
    for buf, off, ln, w, base in ((lo_buf, lo_offs, lens_a, want_a, 0),
                                  (hi_buf, hi_offs, lens_b, want_b, hi0)):
        t = off.astype(np.int64) + ln.astype(np.int64) - 4
        buf[(t[:, None] + np.arange(4)[None, :]).reshape(-1)] = w.view(np.uint8)
        buf[off[::101].astype(np.int64) + 48] ^= 0x10
        d[base:base + buf.size].copy_(torch.from_numpy(buf))
    expect_ok = np.ones(2 * n, bool)
    expect_ok[0::2][::101] = False
    expect_ok[1::2][::101] = False
    flips = torch.from_numpy(np.concatenate(
        [lo_offs[::101].astype(np.int64) + 48, hi_offs[::101].astype(np.int64) + 48 + hi0])).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    s = torch.cuda.current_stream()
    try:
        for lanes in (4, 8, 16):
            engine.set_lanes(lanes)
            out = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
            ok = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
            icrc_v = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
            engine.verify_batch_dev(d, do, dl, 2 * n, ok, icrc_v, stream=s.cuda_stream)
            s.synchronize()
            np.testing.assert_array_equal(ok.cpu().numpy().astype(bool), expect_ok,
                                          err_msg=f"lanes {lanes}")
            d[flips] ^= 0x10  # restore the flipped bits: every computed word bit-exact
            engine.compute_batch_dev(d, do, dl, 2 * n, out, stream=s.cuda_stream)
            s.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want,
                                          err_msg=f"lanes {lanes}")
            d[flips] ^= 0x10
    finally:
        engine.set_lanes(0)
        del d
        torch.cuda.empty_cache()


def test_small_kernel_beyond_4_gib(engine):
    """The lane-per-packet kernel over 42 x 999983 frames of 128 B (5.4 GB,
    stride = the small kernel's maximum): batch and frame addresses cross
    2^32 bytes.  The buffer tiles a prime number of distinct frames, so an
    address that wrapped at 2^32 would read a frame with a different ICRC;
    every word is checked against the tiled C-oracle result."""
    torch = pytest.importorskip("torch")
    m, reps = 999983, 42
    buf, stride, flen = synth.uniform_frames(m, 84, seed=synth.SEED_CFG5)
    assert stride == 128
    want, _ = oracle_batch(buf, stride=stride, length=flen, n=m)
    n = m * reps
    d = torch.from_numpy(buf).cuda().repeat(reps)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.compute_strided_dev(d, stride, flen, n, out, stream=s.cuda_stream)
    s.synchronize()
    got = out.cpu().numpy().view(np.uint32).reshape(reps, m)
    bad = np.nonzero((got != want[None, :]).any(axis=1))[0]
    assert bad.size == 0, f"tiles with wrong words: {bad.tolist()}"
    del d
    torch.cuda.empty_cache()


@pytest.mark.parametrize("lanes", [0, 1, 4, 8, 64])
def test_any_frame_length(engine, lanes):
    """zlib.crc32 takes any length, so does the reference's compute_icrc: frames
    of every length 44 .. 700 B (every residue mod 4) at every byte alignment,
    ragged (host and device) and strided with odd strides, compute and verify
    (trailers = the oracle's words, every 7th with a flipped covered bit)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(4242 + lanes)
    frames = []
    for L in range(44, 701):
        f = bytearray(o.build_frame("10.1.2.3", "10.3.2.1", 77, dict(opcode=0x07, psn=L),
                                    payload=rng.integers(0, 256, L - 44, dtype=np.uint8).tobytes()))
        del f[L:]  # the exact length (a payload of L - 44 bytes was padded to 4)
        f[2:4] = L.to_bytes(2, "big")
        frames.append(bytes(f))
    offs, pos = [], 0
    for i, f in enumerate(frames):
        pos += i % 4  # every byte misalignment in turn
        offs.append(pos)
        pos += len(f)
    buf = np.zeros(pos + 8, np.uint8)
    for off, f in zip(offs, frames):
        buf[off:off + len(f)] = np.frombuffer(f, np.uint8)
    offs = np.array(offs, np.uint64)
    lens = np.array([len(f) for f in frames], np.uint32)
    want = np.array([o.icrc_of_frame(f) for f in frames], np.uint32)
    for i, (a, L) in enumerate(zip(offs, lens)):
        e = int(a + L)
        buf[e - 4:e] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    flip = np.arange(3, len(frames), 7)
    for i in flip:
        buf[int(offs[i]) + 42] ^= 0x10
    want, ok_want = oracle_batch(buf, offs, lens)
    assert (want != 0).all()
    engine.set_lanes(lanes)
    try:
        got, st = engine.compute_batch(buf, offs, lens)
        ok, got2, _ = engine.verify_batch(buf, offs, lens)
        d = torch.from_numpy(buf).cuda()
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        dl = torch.from_numpy(lens.view(np.int32)).cuda()
        dout = torch.zeros(len(frames), dtype=torch.int32, device="cuda")
        engine.compute_batch_dev(d, do, dl, len(frames), dout)
        torch.cuda.synchronize()
    finally:
        engine.set_lanes(0)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got2, want)
    np.testing.assert_array_equal(dout.cpu().numpy().view(np.uint32), want)
    np.testing.assert_array_equal(ok, ok_want.astype(bool))
    assert not ok[flip].any() and ok.sum() == len(frames) - flip.size
    assert not (st & PKT_BAD_LEN).any()
    # strided, every length residue and odd strides (the small-frame kernel
    # takes multiples of 4 only; the rest go through the lane-group kernels)
    for L, stride in ((45, 45), (46, 47), (47, 48), (101, 101), (4139, 4141)):
        n = 1001
        fr = bytearray(o.build_frame("10.1.2.3", "10.3.2.1", 77, dict(opcode=0x01, psn=1),
                                     payload=bytes(range(256)) * ((L - 44) // 256 + 1)))
        del fr[L:]
        fr[2:4] = L.to_bytes(2, "big")
        sb = np.zeros(n * stride, np.uint8)
        rows = np.lib.stride_tricks.as_strided(sb, (n, L), (stride, 1))
        rows[:] = np.frombuffer(bytes(fr), np.uint8)
        rows[:, 40] = np.arange(n, dtype=np.uint8)  # distinct frames (first payload byte)
        w, _ = oracle_batch(sb, stride=stride, length=L, n=n)
        engine.set_lanes(lanes)
        try:
            g, s2 = engine.compute_strided(sb, stride, L, n)
        finally:
            engine.set_lanes(0)
        np.testing.assert_array_equal(g, w, err_msg=f"L {L} stride {stride}")

"""GPU: the golden fixtures and the reference-mirror packet API through the
HIP engine (BTH.compute_icrc / post_build / emit_batch / verify_frames)."""
import json

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

import icrc_oracle as o  # noqa: E402  (checker only)
from roce_icrc import roce as R  # noqa: E402

VEC = json.loads((GOLDEN / "vectors.json").read_text())["vectors"]
BLOB = np.frombuffer((GOLDEN / "frames.bin").read_bytes(), np.uint8)


@pytest.mark.parametrize("lanes", [0, 1, 2, 4, 8, 16, 32, 64])
def test_golden_vectors_on_gpu(engine, lanes):
    offs = np.array([v["offset"] for v in VEC], np.uint64)
    lens = np.array([v["len"] for v in VEC], np.uint32)
    want = np.array([int(v["icrc"], 16) for v in VEC], np.uint32)
    engine.set_lanes(lanes)
    try:
        got, st = engine.compute_batch(BLOB, offs, lens)
    finally:
        engine.set_lanes(0)
    np.testing.assert_array_equal(got, want)
    # frames the reference would not CRC (not IPv4/UDP) carry a fatal status bit
    fatal = np.array([o.masked_pseudo_packet(bytes(BLOB[v["offset"]:v["offset"] + v["len"]]))
                      is None for v in VEC])
    assert fatal.sum() == 3
    assert (st[fatal] & 0x06).all() and not (st[~fatal] & 0x07).any()


def test_bth_post_build_through_engine(engine):
    R.set_engine(engine)
    pkt = R.BTH(opcode=0x04, psn=0, dqpn=0x11, ackreq=1) / R.Raw(load=b"\xff")
    frame = bytes(R.l3_packet(pkt, dst="10.1.1.15", sport=2, src="10.1.1.48"))
    assert frame == o.sim_send_success_frame()
    assert frame[-4:] == bytes.fromhex("751de21b")


def test_ipv4_options_post_build_and_emit_batch(engine):
    """IP(options=...) frames (ihl 6..15) through the engine: BTH.post_build
    (src/roce.py:228-233) and emit_batch give the oracle's frame byte for
    byte, the ICRC over the longer header included; they verify on the GPU."""
    R.set_engine(engine)
    pkts, refs = [], []
    for i, raw in enumerate([b"\x01\x01\x01\x00", b"\x94\x04\x00\x00", b"\x07\x07\x04\x0a\x0b\x0c\x0d",
                             b"\x01" * 40, b"\x83\x0b\x04" + bytes(8)]):
        payload = bytes((i + k) & 0xFF for k in range(13 + 50 * i))
        refs.append(o.build_frame("10.0.0.1", "10.0.0.2", 0x21, dict(opcode=0x0A, psn=i, dqpn=0x21),
                                  ext=o.reth_bytes(i, 7, len(payload)), payload=payload, ip_options=raw))
        b = R.add_padding_if_needed(R.BTH(opcode=0x0A, psn=i, dqpn=0x21) /
                                    R.RETH(va=i, rkey=7, dlen=len(payload)) / R.Raw(load=payload))
        pkts.append(R.IP(src="10.0.0.1", dst="10.0.0.2", options=raw) / R.UDP(dport=4791, sport=0x21) / b)
    assert [bytes(p) for p in pkts] == refs  # one by one: post_build -> ricrc_compute_one
    assert R.emit_batch(pkts) == refs  # one GPU call
    assert R.verify_frames(refs).all()
    got, dropped = R.recv_datagrams(refs)
    assert dropped == [] and [b.psn for b in got] == list(range(5))


def test_emit_batch_and_verify(engine):
    R.set_engine(engine)
    rng = np.random.default_rng(1)
    pkts = []
    for i in range(200):
        op = int(rng.choice([0x00, 0x01, 0x04, 0x06, 0x0A, 0x0D, 0x11, 0x13]))
        b = R.BTH(opcode=op, psn=i, dqpn=0x21, ackreq=i & 1)
        if op in (0x06, 0x0A):
            b = b / R.RETH(va=i, rkey=7, dlen=100)
        elif op in (0x0D, 0x11):
            b = b / R.AETH(code="ACK", value=31, msn=i)
        elif op == 0x13:
            b = b / R.AtomicETH(va=i, rkey=1, swap=2, comp=3)
        if op not in (0x11, 0x13):
            b = b / R.Raw(load=rng.integers(0, 256, int(rng.integers(0, 900)), dtype=np.uint8).tobytes())
        pkts.append(R.l3_packet(b, dst="10.0.0.2", sport=0x21, src="10.0.0.1"))
    frames = R.emit_batch(pkts)
    assert frames[:5] == [bytes(p) for p in pkts[:5]]  # one-by-one post_build path agrees
    for f in frames:
        assert o.verify_frame(f)
    ok = R.verify_frames(frames)
    assert ok.all()
    bad = list(frames)
    bad[3] = bad[3][:50] + bytes([bad[3][50] ^ 0x10]) + bad[3][51:]
    ok = R.verify_frames(bad)
    assert not ok[3] and ok.sum() == len(frames) - 1


def test_recv_datagrams_drops_bad_icrc(engine):
    R.set_engine(engine)
    pkts = [R.l3_packet(R.BTH(opcode=0x01, psn=i, dqpn=0x30 + (i % 2)) / R.Raw(load=bytes([i]) * 64),
                        dst="10.0.0.2", sport=7, src="10.0.0.1") for i in range(10)]
    frames = R.emit_batch(pkts)
    frames[4] = frames[4][:60] + bytes([frames[4][60] ^ 4]) + frames[4][61:]
    got, dropped = R.recv_datagrams(frames)
    assert dropped == [4] and len(got) == 9
    assert [b.psn for b in got] == [0, 1, 2, 3, 5, 6, 7, 8, 9]
    assert got[0][R.Raw].load == bytes([0]) * 64
    got, dropped = R.recv_datagrams(frames, qpn=0x31)
    assert [b.psn for b in got] == [1, 3, 5, 7, 9]


def test_odd_length_datagram_does_not_shift_the_batch(engine):
    """A stray datagram whose length is not a multiple of 4 (truncated UDP
    packet) in the middle of a receive batch: it fails, and every valid frame
    after it still verifies and is delivered (frames are packed at dword-aligned
    offsets).  On the emit side an odd-length frame gets the reference's ICRC
    (zlib.crc32 takes any length; the engine's byte-load path), and the
    frames after it theirs."""
    R.set_engine(engine)
    pkts = [R.l3_packet(R.BTH(opcode=0x01, psn=i, dqpn=0x30) / R.Raw(load=bytes([i]) * 64),
                        dst="10.0.0.2", sport=7, src="10.0.0.1") for i in range(8)]
    frames = R.emit_batch(pkts)
    for cut in (1, 2, 3):
        stray = frames[0][:-cut]  # length not a multiple of 4
        batch = frames[:3] + [stray] + frames[3:]
        ok = R.verify_frames(batch)
        assert list(ok) == [True] * 3 + [False] + [True] * 5
        got, dropped = R.recv_datagrams(batch)
        assert dropped == [3] and [b.psn for b in got] == list(range(8))
    # emit side: a BTH/Raw build without padding gives an odd-length frame
    raw = R.IP(src="10.0.0.1", dst="10.0.0.2") / R.UDP(dport=4791, sport=7) / \
        R.BTH(opcode=0x04, psn=99, dqpn=0x30) / R.Raw(load=b"\x01\x02\x03")
    mixed = R.emit_batch(pkts[:2] + [raw] + pkts[2:])
    assert len(mixed[2]) % 4 == 3 and mixed[:2] + mixed[3:] == frames
    assert mixed[2][-4:] == int(o.icrc_of_frame(mixed[2])).to_bytes(4, "little")
    assert o.verify_frame(mixed[2]) and R.verify_frames([mixed[2]])[0]
    # padded as the reference's emit wrap pads it, the same packet goes through
    padded = R.l3_packet(R.BTH(opcode=0x04, psn=99, dqpn=0x30) / R.Raw(load=b"\x01\x02\x03"),
                         dst="10.0.0.2", sport=7, src="10.0.0.1")
    mixed = R.emit_batch(pkts[:2] + [padded] + pkts[2:])
    assert mixed[:2] + mixed[3:] == frames
    assert len(mixed[2]) % 4 == 0 and o.verify_frame(mixed[2])
    assert mixed[2][-4:] == int(o.icrc_of_frame(mixed[2])).to_bytes(4, "little")
    for f in frames:
        assert o.verify_frame(f)

"""CPU: the oracle (test infrastructure) against the golden fixtures, zlib's
CRC-32 check value, and its independent C restatements."""
import json
import zlib

import numpy as np
import pytest

from conftest import GOLDEN, oracle_batch, oracle_lib

import icrc_oracle as o

VEC = json.loads((GOLDEN / "vectors.json").read_text())["vectors"]
BLOB = (GOLDEN / "frames.bin").read_bytes()


def frame(v):
    return BLOB[v["offset"]:v["offset"] + v["len"]]


def test_zlib_is_crc32_iso_hdlc():
    # the arithmetic the reference calls (src/roce.py:32, 218)
    assert zlib.crc32(b"123456789") == 0xCBF43926
    assert ~zlib.crc32(b"\xff" * 8) & 0xFFFFFFFF == o.ICRC_SEED_REGISTER


def test_config1_worked_example():
    """masked bytes and ICRC of the sim_send_success SEND_ONLY."""
    f = o.sim_send_success_frame()
    assert o.masked_pseudo_packet(f)[8:].hex() == (
        "45ff003000010000ff11ffff0a0101300a01010f000212b7001cffff0430ffffff00001180000000ff000000")
    assert o.icrc_of_frame(f) == 0x1BE21D75
    assert f[-4:] == bytes.fromhex("751de21b")  # little-endian wire bytes (src/roce.py:190)


@pytest.mark.parametrize("v", VEC, ids=[v["name"] for v in VEC])
def test_golden_vector(v):
    f = frame(v)
    want = int(v["icrc"], 16)
    assert o.icrc_of_frame(f) == want
    assert o.icrc_bitwise(f) == want
    assert o.icrc_of_frame_at(f, 0, len(f)) == want
    lib = oracle_lib()
    assert lib.oracle_icrc_bitwise(f, len(f)) == want
    assert lib.oracle_icrc_sliced(f, len(f)) == want


def test_golden_categories():
    by = {}
    for v in VEC:
        by.setdefault(v["kind"], []).append(v)
    base = int(by["mask_base"][0]["icrc"], 16)
    assert all(int(v["icrc"], 16) == base for v in by["mask_variant"])
    assert all(int(v["icrc"], 16) != base for v in by["sensitivity"])
    assert all(int(v["icrc"], 16) == 0 for v in by["warning_path"])
    ops = {v["opcode"] for v in by["opcode"]}
    assert len(ops) == 24  # every RC opcode the simulator can emit + CNP
    pads = {(-v["payload"]) % 4 for v in by["opcode"] if v["payload"] is not None}
    assert pads == {0, 1, 2, 3}


def test_frames_carry_their_icrc():
    for v in VEC:
        if v["kind"] in ("opcode", "config1"):
            assert o.verify_frame(frame(v)), v["name"]


def test_c_batch_matches_python():
    from roce_icrc import synth
    buf, offs, lens = synth.mixed_mtu_frames(300, seed=5)
    got, _ = oracle_batch(buf, offs, lens, nthreads=4)
    want = [o.icrc_of_frame(bytes(buf[int(a):int(a) + int(b)])) for a, b in zip(offs, lens)]
    np.testing.assert_array_equal(got, want)
    buf, stride, flen = synth.uniform_frames(64, 4096, seed=6)
    got, _ = oracle_batch(buf, stride=stride, length=flen, n=64, nthreads=3)
    want = [o.icrc_of_frame(bytes(buf[i * stride:i * stride + flen])) for i in range(64)]
    np.testing.assert_array_equal(got, want)

"""GPU parity of the lane-per-packet kernel for small strided frames
(stride <= 128 B, automatic lanes; strides past 64 B run 32-frame batches with
two lanes per frame, every front pad 0-3 below): batch boundaries, strides with gaps,
IPv4 options (the generic-mask path), malformed frames, verify mode, and
agreement with the lane-group kernels on the same bytes."""
import numpy as np
import pytest

import icrc_oracle as o
from conftest import oracle_batch
from roce_icrc.engine import PKT_BAD_LEN, PKT_ICRC_MISMATCH, PKT_NOT_IPV4

pytestmark = pytest.mark.gpu


def _frame(L, rng, ihl6=False):
    pay = L - 44 - (4 if ihl6 else 0)
    f = bytearray(o.build_frame("10.0.0.1", "10.0.0.2", int(rng.integers(1 << 16)),
                                dict(opcode=0x01, psn=int(rng.integers(1 << 24)), dqpn=0x11),
                                payload=rng.integers(0, 256, pay, dtype=np.uint8).tobytes()))
    if ihl6:  # insert one dword of IPv4 options; lengths follow
        f = f[:20] + bytearray(b"\x01\x01\x01\x00") + f[20:]
        f[0] = 0x46
        f[2:4] = len(f).to_bytes(2, "big")
    assert len(f) == L
    return bytes(f)


def _strided(n, L, stride, rng, ihl6_every=0, bad_every=0):
    buf = np.zeros((n - 1) * stride + L, np.uint8)
    for i in range(n):
        f = _frame(L, rng, ihl6=bool(ihl6_every and i % ihl6_every == 3))
        if bad_every and i % bad_every == 5:
            f = b"\x60" + f[1:]  # IPv6 version nibble -> not IPv4
        buf[i * stride: i * stride + L] = np.frombuffer(f, np.uint8)
    return buf


@pytest.mark.parametrize("n", [1, 2, 31, 32, 33, 63, 64, 65, 255, 257, 1023, 4099])
@pytest.mark.parametrize("L,stride", [(48, 48), (108, 108), (108, 112), (64, 128), (128, 128),
                                      (68, 68), (72, 72), (76, 80), (80, 84), (100, 100), (124, 128)])
def test_small_kernel_matches_oracle(engine, n, L, stride):
    rng = np.random.default_rng(n * 1000 + L + stride)
    buf = _strided(n, L, stride, rng)
    assert engine.lanes_for_len(L) == 1
    got, st = engine.compute_strided(buf, stride, L, n)
    want, _ = oracle_batch(buf, stride=stride, length=L, n=n)
    np.testing.assert_array_equal(got, want)
    assert not st.any()


def test_ipv4_options_and_malformed_frames(engine):
    n, L, stride = 3000, 108, 108
    rng = np.random.default_rng(1)
    buf = _strided(n, L, stride, rng, ihl6_every=7, bad_every=11)
    got, st = engine.compute_strided(buf, stride, L, n)
    want = np.array([o.icrc_of_frame(bytes(buf[i * stride: i * stride + L])) or 0
                     for i in range(n)], np.uint32)
    bad = np.array([i % 11 == 5 for i in range(n)])
    np.testing.assert_array_equal(got[~bad], want[~bad])
    assert (got[bad] == 0).all() and (st[bad] & PKT_NOT_IPV4).all()
    assert not st[~bad].any()


def test_same_result_as_lane_group_kernels(engine):
    n, L = 20000, 108
    rng = np.random.default_rng(2)
    buf = _strided(n, L, L, rng, ihl6_every=13, bad_every=17)
    small, st_small = engine.compute_strided(buf, L, L, n)
    engine.set_lanes(2)
    try:
        grid, st_grid = engine.compute_strided(buf, L, L, n)
    finally:
        engine.set_lanes(0)
    np.testing.assert_array_equal(small, grid)
    np.testing.assert_array_equal(st_small, st_grid)


@pytest.mark.parametrize("n", [64, 1000, 100003])
def test_small_kernel_verify(engine, n):
    import torch
    L = 108
    rng = np.random.default_rng(n)
    buf = _strided(n, L, L, rng)
    icrc, _ = oracle_batch(buf, stride=L, length=L, n=n)
    frames = buf.reshape(n, L)
    frames[:, L - 4:] = icrc.astype("<u4").view(np.uint8).reshape(n, 4)
    flip = rng.choice(n, size=max(1, n // 100), replace=False)
    frames[flip, 50] ^= 0x10
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(buf).to(dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    engine.verify_strided_dev(d, L, L, n, ok, None, st)
    torch.cuda.synchronize()
    okh, sth = ok.cpu().numpy().astype(bool), st.cpu().numpy()
    want = np.ones(n, bool)
    want[flip] = False
    np.testing.assert_array_equal(okh, want)
    assert (sth[flip] & PKT_ICRC_MISMATCH).all() and not sth[want].any()


def _dev_strided(engine, buf, L, n, verify):
    """Device-resident packed batch (stride == L): compute with ICRC words only
    (bench.py's form), or verify with verdicts only and with verdicts + words."""
    import torch
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(buf).to(dev)
    if not verify:
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        engine.compute_strided_dev(d, L, L, n, out)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint32)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    engine.verify_strided_dev(d, L, L, n, ok)
    ok2 = torch.zeros(n, dtype=torch.uint8, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    engine.verify_strided_dev(d, L, L, n, ok2, out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ok.cpu().numpy(), ok2.cpu().numpy())
    return ok.cpu().numpy().astype(bool), out.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("L", list(range(44, 129, 4)))
def test_device_resident_every_packed_length(engine, L):
    """Packed batches (stride == frame length) through the device-resident
    forms: every length 44..128 B (every chunk count and front pad of the
    two-chain fold), batch counts across the 64-packet batch, output-ring and
    last-batch boundaries, compute and both verify forms, against the
    oracle."""
    rng = np.random.default_rng(L)
    for n in (1, 63, 64, 65, 4099, 70001):
        buf = _strided(n, L, L, rng) if n <= 4099 else np.tile(_strided(4099, L, L, rng),
                                                               n // 4099 + 1)[:n * L].copy()
        want, _ = oracle_batch(buf, stride=L, length=L, n=n)
        got = _dev_strided(engine, buf, L, n, verify=False)
        np.testing.assert_array_equal(got, want, err_msg=f"L {L} n {n}")
        frames = buf.reshape(n, L)
        frames[:, L - 4:] = want.astype("<u4").view(np.uint8).reshape(n, 4)
        flip = np.arange(3, n, 37)
        frames[flip, L - 8] ^= 0x01  # the last covered dword: must fail
        ok, words = _dev_strided(engine, buf, L, n, verify=True)
        expect = np.ones(n, bool)
        expect[flip] = False
        np.testing.assert_array_equal(ok, expect, err_msg=f"L {L} n {n}")
        # the words are those of the frames as they are (flipped ones differ)
        np.testing.assert_array_equal(np.delete(words, flip), np.delete(want, flip),
                                      err_msg=f"L {L} n {n}")
        assert (words[flip] != want[flip]).all()


@pytest.mark.parametrize("L", [48, 68, 108, 128])
def test_device_resident_options_and_malformed(engine, L):
    """Batches holding IPv4-option or malformed frames fold from HBM through
    the per-dword masks (the slot already holds the next batch): ICRC words
    against the oracle, malformed frames 0."""
    n = 64 * 50 + 9
    rng = np.random.default_rng(L + 1)
    buf = _strided(n, L, L, rng, ihl6_every=29, bad_every=31)
    want = np.array([o.icrc_of_frame(bytes(buf[i * L:(i + 1) * L])) or 0 for i in range(n)],
                    np.uint32)
    got = _dev_strided(engine, buf, L, n, verify=False)
    np.testing.assert_array_equal(got, want)
    bad = np.array([i % 31 == 5 for i in range(n)])
    assert (got[bad] == 0).all()


@pytest.mark.parametrize("stride", [4, 32, 40, 44, 48])
def test_strides_under_44_bytes(engine, stride):
    """Strides under 44 B hold only unusable frames (shorter than IPv4 + UDP +
    BTH + ICRC): they go to the lane-group kernels (the lane-per-packet kernel
    is instantiated from ceil(stride / 16) = 3 chunks up), which give every
    frame ICRC 0 and the bad-length status, as the oracle does (no ICRC); a
    44-B stride is the lane-per-packet kernel's shortest."""
    n = 1000
    rng = np.random.default_rng(stride)
    if stride >= 44:
        buf = _strided(n, stride, stride, rng)
        want, _ = oracle_batch(buf, stride=stride, length=stride, n=n)
        assert engine.lanes_for_len(stride) == 1
    else:
        buf = rng.integers(0, 256, n * stride, dtype=np.uint8)
        want = np.zeros(n, np.uint32)
        assert engine.lanes_for_len(stride) > 1
    got, st = engine.compute_strided(buf, stride, stride, n)
    np.testing.assert_array_equal(got, want)
    if stride < 44:
        assert (st == PKT_BAD_LEN).all()

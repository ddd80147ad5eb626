"""GPU: tiny frames (ACK / NAK / atomic-ack sized) on the device-resident
ragged path.  The mixed-width ragged kernel sorts frames <= 128 B to the
front of each window and runs them as G = 1 sets (one lane per packet) with
Mul(128) restaged into its G = 4 table half; the rest of the window follows
as G = 4 / G = 8 sets.  Bit-exact against the C oracle in compute and verify
mode, including window sequences that switch the table half back and forth."""
import numpy as np
import pytest

from conftest import oracle_batch

pytestmark = pytest.mark.gpu

from roce_icrc import synth  # noqa: E402


def _ragged(lens, seed):
    """Frames of the given lengths (RDMA_WRITE_MIDDLE-shaped, random payload,
    correct headers), packed back to back at dword-aligned offsets."""
    rng = np.random.default_rng(seed)
    lens = np.asarray(lens, np.uint32)
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, int(lens.astype(np.uint64).sum()), dtype=np.uint8)
    tm = {}
    for L in np.unique(lens):
        tm[int(L)] = synth.header_template(int(L) - 44, 0x11)
    for L, t in tm.items():
        sel = np.flatnonzero(lens == L)
        for c in range(0, sel.size, 1 << 16):  # (bounded index temporaries)
            base = offs[sel[c:c + (1 << 16)]].astype(np.int64)
            buf[base[:, None] + np.arange(40)[None, :]] = t
    return buf, offs, lens


def _run(engine, buf, offs, lens, verify=False, flip_every=0):
    torch = pytest.importorskip("torch")
    n = lens.size
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.compute_batch_dev(d, do, dl, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32).copy()
    if not verify:
        return got, None
    # trailers from the GPU words, every flip_every-th frame corrupted
    tr = (do + dl.to(torch.int64) - 4)
    idx = tr[:, None] + torch.arange(4, device="cuda")[None, :]
    d[idx.reshape(-1)] = out.view(torch.uint8).reshape(-1)
    bad = np.arange(0, n, flip_every) if flip_every else np.array([], np.int64)
    if bad.size:
        pos = torch.from_numpy((offs[bad] + 40).astype(np.int64)).cuda()
        d[pos] ^= 1
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch_dev(d, do, dl, n, ok)
    torch.cuda.synchronize()
    return got, (ok.cpu().numpy().astype(bool), bad)


def test_ack_sized_batch_device_resident(engine):
    n = 1 << 18
    rng = np.random.default_rng(1)
    lens = rng.choice([44, 48, 48, 48, 56, 64, 72, 96, 124, 128], n).astype(np.uint32)
    buf, offs, lens = _ragged(lens, 2)
    want, _ = oracle_batch(buf, offs, lens)
    got, (ok, bad) = _run(engine, buf, offs, lens, verify=True, flip_every=101)
    np.testing.assert_array_equal(got, want)
    expect = np.ones(n, bool)
    expect[bad] = False
    np.testing.assert_array_equal(ok, expect)


def test_tiny_and_long_frames_in_one_window(engine):
    """Phase A (tiny frames) and phase B (the rest) in the same windows; also
    a batch whose tiny frames are too few for phase A."""
    rng = np.random.default_rng(3)
    for n, tiny_frac in ((200000, 0.5), (200000, 0.9), (200000, 0.005), (3000, 0.3)):
        big = rng.integers(33, 1100, n) * 4
        small = rng.integers(11, 33, n) * 4
        lens = np.where(rng.random(n) < tiny_frac, small, big).astype(np.uint32)
        buf, offs, lens = _ragged(lens, int(n * tiny_frac * 10))
        want, _ = oracle_batch(buf, offs, lens)
        got, (ok, bad) = _run(engine, buf, offs, lens, verify=True, flip_every=97)
        np.testing.assert_array_equal(got, want, err_msg=f"n {n} tiny {tiny_frac}")
        expect = np.ones(n, bool)
        expect[bad] = False
        np.testing.assert_array_equal(ok, expect)


def test_window_sequences_switch_the_table_half(engine):
    """Three 8192-packet windows per workgroup: tiny-only, mixed, tiny-only
    (Mul(128) staged, Mul(512) restaged, Mul(128) again)."""
    per_wg, W = 3 * 8192, 8192
    wgs = 256
    n = per_wg * wgs
    rng = np.random.default_rng(9)
    t = np.arange(n) % per_wg
    win = t // W
    lens = np.where(win == 1, rng.integers(11, 400, n) * 4, rng.integers(11, 33, n) * 4).astype(np.uint32)
    buf, offs, lens = _ragged(lens, 10)
    want, _ = oracle_batch(buf, offs, lens)
    got, _ = _run(engine, buf, offs, lens)
    np.testing.assert_array_equal(got, want)

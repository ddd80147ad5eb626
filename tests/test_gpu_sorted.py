"""GPU: the SORTED ragged kernel (icrc_ragged_mixed_kernel, mixed_windows) at
the shapes its window logic branches on.  Bit-exact against the C oracle
(src/roce.py:192-223) in compute and verify mode (every verdict byte written,
corrupted frames fail), with status bytes: batches of one and several sort
windows per workgroup, ranges shorter than a wave, tiny (ACK-sized) frames
sorted into the windows with MTU frames, frames stored in shuffled order, and
offsets past 2^34 (which do not fit the sort's offset / 4 word, so the sets
read offsets[i] again).  (Written in round 6 for a tail pool of the sorted
kernel that was measured slower and not kept: scratch/attic/
sorted_tail_pool_r06.diff)"""
import numpy as np
import pytest

from conftest import oracle_batch

pytestmark = pytest.mark.gpu

from roce_icrc import engine as E  # noqa: E402
from roce_icrc import synth  # noqa: E402


def _sorted_run(engine, buf, offs, lens, flip_every=0, status=False):
    torch = pytest.importorskip("torch")
    n = lens.size
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda") if status else None
    engine.set_ragged_variant(E.RAGGED_SORTED)
    try:
        engine.compute_batch_dev(d, do, dl, n, out, st)
        assert engine.last_ragged_variant() == E.RAGGED_SORTED
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32).copy()
        sts = st.cpu().numpy() if status else None
        # trailers from the words, every flip_every-th frame corrupted, verify
        tr = do + dl.to(torch.int64) - 4
        idx = tr[:, None] + torch.arange(4, device="cuda")[None, :]
        d[idx.reshape(-1)] = out.view(torch.uint8).reshape(-1)
        bad = np.arange(3, n, flip_every) if flip_every else np.array([], np.int64)
        if bad.size:
            d[torch.from_numpy((offs[bad] + 41).astype(np.int64)).cuda()] ^= 4
        ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        engine.verify_batch_dev(d, do, dl, n, ok)
        torch.cuda.synchronize()
        okh = ok.cpu().numpy()
    finally:
        engine.set_ragged_variant(E.RAGGED_AUTO)
    assert set(np.unique(okh)) <= {0, 1}, "a verdict byte was never written"
    expect = np.ones(n, bool)
    expect[bad] = False
    np.testing.assert_array_equal(okh.astype(bool), expect)
    return got, sts


@pytest.mark.parametrize("n", [40, 64 * 256 + 9, 200003, 1 << 20])
def test_sorted_mixed_mtu(engine, n):
    buf, offs, lens = synth.mixed_mtu_frames(n, seed=n)
    want, _ = oracle_batch(buf, offs, lens)
    got, st = _sorted_run(engine, buf, offs, lens, flip_every=97, status=True)
    np.testing.assert_array_equal(got, want)
    assert not st.any()


@pytest.mark.timeout(300)
def test_sorted_several_windows_per_workgroup(engine):
    """2^22 + 77 short mixed frames: 16 K packets per workgroup, two sort
    windows each."""
    n = (1 << 22) + 77
    buf, offs, lens = synth.mixed_mtu_frames(n, mtus=(256, 512), seed=5)
    want, _ = oracle_batch(buf, offs, lens)
    got, _ = _sorted_run(engine, buf, offs, lens, flip_every=1001)
    np.testing.assert_array_equal(got, want)


def test_sorted_tiny_frames_and_shuffled_order(engine):
    """ACK-sized and MTU frames mixed (tiny frames sorted to the windows'
    front, phase A), stored in shuffled order (offsets not monotone)."""
    rng = np.random.default_rng(11)
    n = 300001
    buf, offs, lens = synth.mixed_mtu_frames(n, mtus=(4, 8, 256, 1024, 4096), seed=12)
    perm = rng.permutation(n)
    offs, lens = offs[perm].copy(), lens[perm].copy()
    want, _ = oracle_batch(buf, offs, lens)
    got, _ = _sorted_run(engine, buf, offs, lens, flip_every=89)
    np.testing.assert_array_equal(got, want)


def test_sorted_offsets_beyond_2_34(engine):
    """Offsets past 2^34 do not fit the sort's offset / 4 word: the sorted
    descriptors carry the 'no offset' mark and the set reads offsets[i]."""
    torch = pytest.importorskip("torch")
    n = 70000
    buf, offs, lens = synth.mixed_mtu_frames(n, mtus=(256, 512), seed=21)
    want, _ = oracle_batch(buf, offs, lens)
    base = (1 << 34) + 4096
    if torch.cuda.get_device_properties(0).total_memory < base + buf.size + (1 << 30):
        pytest.skip("needs > 17 GB of device memory")
    big = torch.zeros(base + buf.size, dtype=torch.uint8, device="cuda")
    big[base:] = torch.from_numpy(buf).cuda()
    do = torch.from_numpy((offs + np.uint64(base)).view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.set_ragged_variant(E.RAGGED_SORTED)
    try:
        engine.compute_batch_dev(big, do, dl, n, out)
        torch.cuda.synchronize()
    finally:
        engine.set_ragged_variant(E.RAGGED_AUTO)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    del big


# Workgroup-range shapes (round 6, written for byte-balanced ranges, which
# were measured slower and not kept: scratch/attic/sorted_byte_balance_r06.diff,
# DESIGN.md section 12): ranges of very unequal bytes, offsets out of order in
# places, repeated frames, descending offsets.  Every packet must be covered
# exactly once: every word and every verdict byte is checked.

def test_balanced_ranges_skewed_lengths(engine):
    """Buffer-order frames, the first 40 % of 4 KiB MTU, the rest 256-B
    payloads: workgroup ranges of very unequal bytes."""
    n = 1 << 20
    k = n * 2 // 5
    b1, o1, l1 = synth.mixed_mtu_frames(k, mtus=(4096,), seed=31)
    b2, o2, l2 = synth.mixed_mtu_frames(n - k, mtus=(256,), seed=32)
    buf = np.concatenate([b1, b2])
    offs = np.concatenate([o1, o2 + np.uint64(b1.size)])
    lens = np.concatenate([l1, l2])
    want, _ = oracle_batch(buf, offs, lens)
    got, st = _sorted_run(engine, buf, offs, lens, flip_every=997, status=True)
    np.testing.assert_array_equal(got, want)
    assert not st.any()


def test_balanced_ranges_local_swaps_and_duplicates(engine):
    """Buffer order broken by scattered swaps of neighbours, and runs of
    descriptors that repeat one frame (equal offsets)."""
    rng = np.random.default_rng(41)
    n = 600011
    buf, offs, lens = synth.mixed_mtu_frames(n, seed=42)
    offs, lens = offs.copy(), lens.copy()
    for i in rng.choice(n - 1, 700, replace=False):
        offs[[i, i + 1]] = offs[[i + 1, i]]
        lens[[i, i + 1]] = lens[[i + 1, i]]
    for i in rng.choice(n - 8, 300, replace=False):
        offs[i:i + 4] = offs[i]
        lens[i:i + 4] = lens[i]
    want, _ = oracle_batch(buf, offs, lens)
    got, _ = _sorted_run(engine, buf, offs, lens)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("n", [256 * 1024 + 5, 400009])
def test_balanced_ranges_descending_and_short_ranges(engine, n):
    """Offsets in ascending and in descending order, ~1024-1600 packets per
    workgroup."""
    buf, offs, lens = synth.mixed_mtu_frames(n, seed=n + 1)
    want, _ = oracle_batch(buf, offs, lens)
    got, _ = _sorted_run(engine, buf, offs, lens, flip_every=313)
    np.testing.assert_array_equal(got, want)
    r = np.arange(n)[::-1]
    got, _ = _sorted_run(engine, buf, offs[r].copy(), lens[r].copy(), flip_every=313)
    np.testing.assert_array_equal(got, want[r])

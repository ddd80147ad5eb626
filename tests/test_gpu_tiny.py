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

from roce_icrc import engine as E  # noqa: E402
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


VARIANTS = (E.RAGGED_COMPACT, E.RAGGED_SORTED)


def _run(engine, buf, offs, lens, verify=False, flip_every=0):
    """Every launch under both ragged-kernel variants, chosen explicitly
    (ricrc_ctx_set_ragged_variant): the kernel with the compact tiny-batch
    phase and the one without must give the same words and verdicts, and each
    launch must report the variant it was asked for -- whatever ran before on
    the (session-scoped) engine."""
    torch = pytest.importorskip("torch")
    n = lens.size
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    words = []
    try:
        for v in VARIANTS:
            engine.set_ragged_variant(v)
            out.zero_()
            engine.compute_batch_dev(d, do, dl, n, out)
            assert engine.last_ragged_variant() == v
            torch.cuda.synchronize()
            words.append(out.cpu().numpy().view(np.uint32).copy())
    finally:
        engine.set_ragged_variant(E.RAGGED_AUTO)
    np.testing.assert_array_equal(words[0], words[1])
    got = words[0]
    out.copy_(torch.from_numpy(got.view(np.int32)))
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
    oks = []
    try:
        for v in VARIANTS:
            engine.set_ragged_variant(v)
            ok.zero_()
            engine.verify_batch_dev(d, do, dl, n, ok)
            assert engine.last_ragged_variant() == v
            torch.cuda.synchronize()
            oks.append(ok.cpu().numpy().astype(bool))
    finally:
        engine.set_ragged_variant(E.RAGGED_AUTO)
    np.testing.assert_array_equal(oks[0], oks[1])
    return got, (oks[0], bad)


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


def _dev_compute(engine, buf, offs, lens, variant=E.RAGGED_COMPACT):
    """compute_batch_dev with status: (icrc, status) as numpy, on the ragged
    kernel variant asked for (default: the compact kernel, whose
    tests these are -- independent of what the engine ran before)."""
    torch = pytest.importorskip("torch")
    n = lens.size
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.set_ragged_variant(variant)
    try:
        engine.compute_batch_dev(d, do, dl, n, out, st)
        assert engine.last_ragged_variant() == variant
    finally:
        engine.set_ragged_variant(E.RAGGED_AUTO)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32).copy(), st.cpu().numpy().copy()


def test_compact_ack_batches(engine):
    """The compact kernel's groups: packed runs of ACK-sized frames (64
    consecutive packets in order inside 4 KiB) are staged and folded
    lane-per-packet without a sort.  All-ACK batches with a partial last
    group and many groups per wave, plus 44-64 B mixes; compute and verify
    (corrupted trailers and payloads flagged) against the oracle, on both
    variants."""
    rng = np.random.default_rng(21)
    for n, choices in ((100003, [48]), (1 << 22, [48]), (300001, [44, 48, 52, 56, 60, 64])):
        lens = rng.choice(choices, n).astype(np.uint32)
        buf, offs, lens = _ragged(lens, n % 1000)
        want, _ = oracle_batch(buf, offs, lens)
        got, (ok, bad) = _run(engine, buf, offs, lens, verify=True, flip_every=89)
        np.testing.assert_array_equal(got, want, err_msg=f"n {n}")
        expect = np.ones(n, bool)
        expect[bad] = False
        np.testing.assert_array_equal(ok, expect, err_msg=f"n {n}")


def test_compact_batches_malformed_and_options(engine):
    """Frames inside compact groups that leave the IHL-5 fast path: IPv4
    options (IHL 6), not IPv4, not UDP, a wrong IP total length.  ICRC words
    against the oracle on both variants, and status bits against the
    sorted lane-group kernel on the same frames."""
    from roce_icrc import IcrcEngine
    import icrc_oracle as o  # checker only
    n = 64 * 300 + 17
    rng = np.random.default_rng(5)
    lens = np.full(n, 48, np.uint32)
    frames = []
    for i in range(n):
        if i % 97 == 5:  # IHL 6: one option dword, 52 B
            f = bytearray(o.build_frame("10.0.0.1", "10.0.0.2", 7, dict(opcode=0x11, psn=i),
                                        ext=o.aeth_bytes()))
            f = f[:20] + bytearray(b"\x01\x01\x01\x01") + f[20:]
            f[0] = 0x46
            tot = len(f)
            f[2:4] = tot.to_bytes(2, "big")
            frames.append(bytes(f))
            continue
        f = bytearray(o.build_frame("10.0.0.1", "10.0.0.2", 7, dict(opcode=0x11, psn=i),
                                    ext=o.aeth_bytes()))
        if i % 89 == 3:
            f[0] = 0x65           # not IPv4
        elif i % 83 == 7:
            f[9] = 6              # TCP
        elif i % 79 == 1:
            f[3] ^= 4             # IP total length mismatch
        f[-4:] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        frames.append(bytes(f))
    from roce_icrc import pack_aligned
    buf, offs, lens = pack_aligned(frames)
    want = np.array([o.icrc_of_frame(f) for f in frames], np.uint32)
    got, st = _dev_compute(engine, buf, offs, lens)
    np.testing.assert_array_equal(got, want)
    got_s, st_s = _dev_compute(engine, buf, offs, lens, E.RAGGED_SORTED)
    np.testing.assert_array_equal(got_s, want)
    np.testing.assert_array_equal(st_s, st)
    e8 = IcrcEngine(0, lanes=8)
    try:
        got8, st8 = _dev_compute(e8, buf, offs, lens, E.RAGGED_SORTED)
    finally:
        e8.close()
    np.testing.assert_array_equal(got8, want)
    np.testing.assert_array_equal(st, st8)
    assert (st != 0).sum() > 100


def test_compact_test_rejects_unsafe_layouts(engine):
    """Groups the compact test must NOT take (the compact kernel folds them by
    lane groups, still exact): frames in reverse order, the same frame twice
    (in-place masks would be applied twice), a gap that stretches the span
    past 4 KiB, frames at 2-byte offsets, and frames longer than 128 B
    between tiny ones -- on both variants."""
    rng = np.random.default_rng(8)
    n = 64 * 64
    lens = np.full(n, 48, np.uint32)
    buf, offs, lens = _ragged(lens, 4)
    offs = offs.copy()
    b = lambda k: slice(64 * k, 64 * k + 64)  # noqa: E731
    offs[b(1)] = offs[b(1)][::-1].copy()                      # reversed
    offs[b(2)][10] = offs[b(2)][9]                            # duplicate frame
    offs[b(3)][32:] += 4096                                   # gap: span > 4 KiB
    big = np.zeros(buf.size + 8192 + 4096, np.uint8)
    big[:buf.size] = buf
    buf = big
    # 2-byte-offset copy of batch 4's frames at the end of the buffer
    src = offs[b(4)].astype(np.int64)
    dst = buf.size - 4096 + 2 + 48 * np.arange(64)
    for s_, d_ in zip(src, dst):
        buf[d_:d_ + 48] = buf[s_:s_ + 48]
    offs[b(4)] = dst.astype(np.uint64)
    want, _ = oracle_batch(buf, offs, lens)
    for v in VARIANTS:
        got, _ = _dev_compute(engine, buf, offs, lens, v)
        np.testing.assert_array_equal(got, want)
    # a 300-B frame between ACKs: that batch is not compact, its neighbours are
    lens2 = np.full(n, 48, np.uint32)
    lens2[64 * 5 + 7] = 300
    buf2, offs2, lens2 = _ragged(lens2, 6)
    want2, _ = oracle_batch(buf2, offs2, lens2)
    for v in VARIANTS:
        got2, _ = _dev_compute(engine, buf2, offs2, lens2, v)
        np.testing.assert_array_equal(got2, want2)


def test_compact_rounds_between_sorted_rounds(engine):
    """64-packet blocks that are all ACK-sized or all longer frames, chosen
    per block: the compact kernel's waves alternate between compact groups
    and lane-group fallback groups with their spans in flight across both
    (and the sorted kernel sorts the same windows); runs of compact groups
    only; blocks shifted by 32 packets (no group compact); a partial last
    group.  Compute and verify (flipped frames fail) against the oracle."""
    rng = np.random.default_rng(31)
    for n, shift, p_ack in ((8192 * 40 + 777, 0, 0.5), (8192 * 24 + 64 * 5, 0, 0.97),
                            (8192 * 12 + 100, 32, 0.5)):
        nb = (n + shift + 63) // 64
        ack = rng.random(nb) < p_ack
        blk = (np.arange(n) + shift) // 64
        tiny = rng.choice([44, 48, 48, 48, 52, 64], n)  # (64 of them fit in 4 KiB)
        big = rng.integers(33, 1100, n) * 4
        lens = np.where(ack[blk], tiny, big).astype(np.uint32)
        buf, offs, lens = _ragged(lens, n % 997)
        want, _ = oracle_batch(buf, offs, lens)
        got, (ok, bad) = _run(engine, buf, offs, lens, verify=True, flip_every=83)
        np.testing.assert_array_equal(got, want, err_msg=f"n {n} shift {shift}")
        expect = np.ones(n, bool)
        expect[bad] = False
        np.testing.assert_array_equal(ok, expect, err_msg=f"n {n} shift {shift}")


def test_bench_ack_workload_line():
    """bench.py --workload ack (device-resident ragged ACK frames, the compact
    tiny-batch phase): the line's device check and per-rank sampled parity
    pass; SURVEY 8(d)'s roofline accounting (frame + word, the 12-B
    descriptors reported apart); every timed launch on the compact kernel."""
    import json
    import os
    import subprocess
    import sys
    from conftest import ROOT
    cmd = [sys.executable, str(ROOT / "bench.py"), "--workload", "ack", "--packets", "300000",
           "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-e2e"]
    r = subprocess.run(cmd, cwd=str(ROOT), capture_output=True, text=True, timeout=300,
                       env=dict(os.environ))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["checks"]["pass"] and d["config"]["packets_per_gpu"] == 300000
    assert all(m == 0 for m in d["parity"]["mismatches_per_rank"])
    assert d["roofline"]["alg_bytes_per_launch"] == 300000 * (44 + 4)
    assert d["roofline"]["descriptor_bytes_per_launch"] == 300000 * 12
    assert d["config"]["ragged_kernel"].startswith("compact")


def test_kernel_choice_follows_the_frames():
    """AUTO on device-resident batches: a fresh context's first ragged launch
    runs the sorted kernel (no hint yet); after ACK frames the next runs the
    compact one, after a batch without tiny frames the next runs the sorted
    one again -- every word bit-exact either way (cfg3-shaped frames, ACK
    frames, alternating)."""
    torch = pytest.importorskip("torch")
    from roce_icrc import IcrcEngine, synth
    eng = IcrcEngine(0)
    try:
        cases = []
        buf, offs, lens = synth.mixed_mtu_frames(20000, seed=7)
        cases.append((buf, offs, lens))
        buf, offs, lens = synth.mixed_mtu_frames(60000, mtus=(4,), opcode=0x11, seed=8)
        cases.append((buf, offs, lens))
        for buf, offs, lens in cases + cases + cases[::-1]:
            want, _ = oracle_batch(buf, offs, lens)
            got, _ = _run(eng, buf, offs, lens)
            np.testing.assert_array_equal(got, want)
    finally:
        eng.close()



def test_variant_named_per_launch_when_batches_alternate():
    """ABI 5: a context whose device-resident batches alternate composition --
    mixed-MTU data (src/roce_v2.py:327-372) and packed ACK runs
    (src/roce_rq.py:767-853) -- names the ragged variant per call.  Launches
    enqueued back to back without a synchronisation each run the variant
    named (ricrc_ctx_last_ragged_variant), every word bit-exact.  (Their
    speeds are bench evidence, not a correctness gate: scripts/perf_ratios.py
    times the ACK batch on both variants, profiles/r06/perf_ratios_*.json.)"""
    torch = pytest.importorskip("torch")
    from roce_icrc import IcrcEngine
    eng = IcrcEngine(0)
    try:
        data = synth.mixed_mtu_frames(20000, seed=7)
        ack = synth.mixed_mtu_frames(1 << 22, mtus=(4,), opcode=0x11, seed=8)
        dev = []
        for buf, offs, lens in (data, ack):
            dev.append((torch.from_numpy(buf).cuda(), torch.from_numpy(offs.view(np.int64)).cuda(),
                        torch.from_numpy(lens.view(np.int32)).cuda(), lens.size))
        want = [oracle_batch(*data)[0], oracle_batch(*ack)[0]]
        plan = [(0, E.RAGGED_SORTED), (1, E.RAGGED_COMPACT)] * 3 + [(1, E.RAGGED_SORTED),
                                                                     (0, E.RAGGED_COMPACT)]
        outs, ran = [], []
        s = torch.cuda.current_stream()
        for which, v in plan:
            d, do, dl, n = dev[which]
            out = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.set_ragged_variant(v)
            eng.compute_batch_dev(d, do, dl, n, out, stream=s.cuda_stream)
            ran.append(eng.last_ragged_variant())
            outs.append(out)
        torch.cuda.synchronize()
        assert ran == [v for _, v in plan]
        for (which, v), out in zip(plan, outs):
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want[which],
                                          err_msg=f"batch {which} variant {v}")
    finally:
        eng.close()


def _ack_stream(n, seed):
    """n 48-B ACK frames (IPv4/UDP/BTH/AETH, src/roce_rq.py:767-776) packed back
    to back, PSN = i, random AETH; built row-wise (fast at 2^24 frames)."""
    rng = np.random.default_rng(seed)
    rows = np.empty((n, 48), np.uint8)
    rows[:, :40] = synth.header_template(4, 0x11)
    psn = np.arange(n, dtype=np.uint32)
    rows[:, 37], rows[:, 38], rows[:, 39] = psn >> 16, psn >> 8, psn
    rows[:, 40:44] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    rows[:, 44:] = 0
    offs = np.arange(n, dtype=np.uint64) * np.uint64(48)
    return rows.reshape(-1), offs, np.full(n, 48, np.uint32)


@pytest.mark.timeout(300)
def test_compact_kernel_second_chunk_of_a_workgroup(engine):
    """The compact kernel's multi-chunk path (advisor, round 5): a workgroup
    whose static range holds more than kCompactChunk = 1024 groups works it in
    chunks, each with its own deferred list (double-buffered counters, the
    list reused, fallback groups folded between chunk barriers).  2^24-odd ACK
    frames give every workgroup 1026 groups; groups made non-compact (two
    frames' descriptors swapped: out of order) sit in the first chunk, at its
    last group, and in the second chunk of several workgroups, and in runs of
    one chunk.  Compute and verify against the oracle, on both variants."""
    torch = pytest.importorskip("torch")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    per_block = 1026
    n = 64 * per_block * cus
    buf, offs, lens = _ack_stream(n, 41)
    bad = []
    for b in sorted({0, 1, cus // 3, cus - 1}):
        bad += [b * per_block + g for g in (0, 5, 1023, 1024, 1025)]
    bad += [3 * per_block + g for g in range(100, 160)]  # a run in one chunk
    for g in bad:
        i, j = 64 * g + 3, 64 * g + 7
        offs[i], offs[j] = offs[j], offs[i]
    assert per_block > 1024 and (n + 63) // 64 == per_block * cus
    want, _ = oracle_batch(buf, offs, lens)
    got, (ok, flipped) = _run(engine, buf, offs, lens, verify=True, flip_every=4099)
    np.testing.assert_array_equal(got, want)
    expect = np.ones(n, bool)
    expect[flipped] = False
    np.testing.assert_array_equal(ok, expect)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 64 * 12 * 8 - 1, 64 * 12 * 8 + 1, 64 * 12 * 16 * 3 + 100,
                               64 * 256 * 12 * 8 + 5 * 64 + 3])
def test_compact_output_ring_edges(engine, n):
    """The compact kernel's output ring (round 6: 16 rounds of words per wave in
    registers, 8-group turns, flushed back to back): batches whose group count
    leaves partial turns, partial rings and a last partial group, with and
    without status bytes (icrc only: the ring; icrc + status: the ring and
    per-group status stores), against the oracle."""
    torch = pytest.importorskip("torch")
    buf, offs, lens = _ack_stream(n, n)
    want, _ = oracle_batch(buf, offs, lens)
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    engine.set_ragged_variant(E.RAGGED_COMPACT)
    try:
        for with_status in (False, True):
            out = torch.full((n + 64,), -1, dtype=torch.int32, device="cuda")
            st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda") if with_status else None
            engine.compute_batch_dev(d, do, dl, n, out, st)
            assert engine.last_ragged_variant() == E.RAGGED_COMPACT
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            np.testing.assert_array_equal(got[:n], want, err_msg=f"status {with_status}")
            assert (got[n:] == 0xFFFFFFFF).all(), "a word was written past the batch"
            if with_status:
                assert not st.cpu().numpy().any()
    finally:
        engine.set_ragged_variant(E.RAGGED_AUTO)

"""GPU ICRC fault injection (ricrc_inject_faults_dev) and the ICRC error
hooks: the selection equals a restatement of its hash, only the allowed bytes
change, and the verify kernel's verdict is exactly the expected one."""
import numpy as np
import pytest

import icrc_oracle as O
from roce_icrc import engine as E
from roce_icrc import hooks as H
from roce_icrc import roce as R
from roce_icrc import synth

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def expected_kinds(seed, n, rate, kinds, usable):
    """Restatement of the selection documented in include/roce_icrc.h."""
    en = [k for k in (1, 2, 4) if kinds & k]
    out = np.zeros(n, np.uint8)
    for i in range(n):
        h = splitmix64(seed ^ ((i * 0xD1B54A32D192ED03) & M64))
        if usable[i] and h % 1000000 < rate and en:
            out[i] = en[(h >> 20) % len(en)]
    return out


def _batch(torch, n, seed=5):
    buf, offs, lens = synth.mixed_mtu_frames(n, seed=seed)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(buf).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    return buf, offs, lens, d, d_offs, d_lens


def _fill_trailers(engine, torch, d, d_offs, d_lens, n):
    icrc = torch.zeros(n, dtype=torch.int32, device=d.device)
    engine.compute_batch_dev(d, d_offs, d_lens, n, icrc)
    trail = d_offs + d_lens.to(torch.int64) - 4
    idx = trail[:, None] + torch.arange(4, device=d.device)[None, :]
    d[idx.reshape(-1)] = icrc.view(torch.uint8).reshape(-1)
    torch.cuda.synchronize()


@pytest.mark.parametrize("kinds", [7, 1, 2, 4])
def test_selection_bytes_and_verdict(engine, kinds):
    import torch
    n, seed, rate = 6000, 0xC0FFEE + kinds, 250000
    buf, offs, lens, d, d_offs, d_lens = _batch(torch, n)
    _fill_trailers(engine, torch, d, d_offs, d_lens, n)
    before = d.cpu().numpy().copy()
    fault = torch.zeros(n, dtype=torch.uint8, device=d.device)
    engine.inject_faults_dev(d, d_offs, d_lens, n, seed, rate, kinds, fault)
    ok = torch.zeros(n, dtype=torch.uint8, device=d.device)
    engine.verify_batch_dev(d, d_offs, d_lens, n, ok)
    torch.cuda.synchronize()
    got = fault.cpu().numpy()
    assert np.array_equal(got, expected_kinds(seed, n, rate, kinds, np.ones(n, bool)))
    assert 0.2 < (got != 0).mean() < 0.3
    after = d.cpu().numpy()
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        a, b = before[o:o + L], after[o:o + L]
        diff = np.nonzero(a != b)[0]
        if got[i] == 0:
            assert diff.size == 0
        elif got[i] == E.FAULT_ICRC:
            assert diff.size == 1 and diff[0] >= L - 4
            assert bin(int(a[diff[0]] ^ b[diff[0]])).count("1") == 1
        elif got[i] == E.FAULT_PAYLOAD:
            assert diff.size == 1 and diff[0] < L - 4
            assert diff[0] not in (1, 8, 10, 11, 26, 27, 32)
            assert bin(int(a[diff[0]] ^ b[diff[0]])).count("1") == 1
        else:
            assert set(diff.tolist()) <= {1, 8, 10, 11, 26, 27, 32}
            assert O.icrc_of_frame(bytes(b)) == O.icrc_of_frame(bytes(a))
    want_ok = ~np.isin(got, [E.FAULT_ICRC, E.FAULT_PAYLOAD])
    assert np.array_equal(ok.cpu().numpy().astype(bool), want_ok)


def test_rate_bounds_and_reproducibility(engine):
    import torch
    n = 3000
    buf, offs, lens, d, d_offs, d_lens = _batch(torch, n, seed=9)
    before = d.clone()
    f0 = torch.zeros(n, dtype=torch.uint8, device=d.device)
    engine.inject_faults_dev(d, d_offs, d_lens, n, 1, 0, 7, f0)
    torch.cuda.synchronize()
    assert int(f0.sum()) == 0 and torch.equal(d, before)
    f1 = torch.zeros(n, dtype=torch.uint8, device=d.device)
    engine.inject_faults_dev(d, d_offs, d_lens, n, 1, 1000000, E.FAULT_ICRC, f1)
    engine.inject_faults_dev(d, d_offs, d_lens, n, 1, 1000000, E.FAULT_ICRC, f1)
    torch.cuda.synchronize()
    assert bool((f1 == E.FAULT_ICRC).all())
    assert torch.equal(d, before)  # the same flips twice cancel
    with pytest.raises(E.IcrcError):
        engine.inject_faults_dev(d, d_offs, d_lens, n, 1, 1000001, 7)


def test_malformed_frames_never_hit(engine):
    import torch
    frames = [b"\x60" + bytes(63), bytes(20), O.sim_send_success_frame()]
    offs = np.array([0, 64, 96], np.uint64)
    lens = np.array([64, 20, len(frames[2])], np.uint32)
    buf = np.frombuffer(b"".join([frames[0], frames[1] + bytes(12), frames[2]]), np.uint8).copy()
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(buf).to(dev)
    fault = torch.zeros(3, dtype=torch.uint8, device=dev)
    engine.inject_faults_dev(d, torch.from_numpy(offs.view(np.int64)).to(dev),
                             torch.from_numpy(lens.view(np.int32)).to(dev), 3, 4, 1000000, 7,
                             fault)
    torch.cuda.synchronize()
    assert fault.cpu().tolist()[:2] == [0, 0] and fault.cpu().tolist()[2] != 0


def test_error_hooks_make_receive_drop(engine):
    R.set_engine(engine)
    hook = H.make_icrc_error_send_hook([2, 4])
    pkts = []
    for psn in range(6):
        ssn, p, _ = hook(0, R.BTH(opcode=0x01, psn=psn, dqpn=9) / R.Raw(load=bytes(range(32))), True)
        pkts.append(R.l3_packet(p, dst="10.1.1.15", sport=3, src="10.1.1.48"))
    frames = R.emit_batch(pkts)
    assert list(R.verify_frames(frames)) == [True, True, False, True, False, True]
    single = bytes(pkts[2])  # per-packet build path (BTH.post_build) honours the mark too
    assert single == frames[2] and not O.verify_frame(single)
    got, dropped = R.recv_datagrams(frames)
    assert dropped == [2, 4] and [b.psn for b in got] == [0, 1, 3, 5]
